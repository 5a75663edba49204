set -e
python tools/fib_churn.py --no-per-route --rate 10000 --period-ms 1 > gpurun_out/churn_1ms.json 2>/dev/null
python tools/fib_churn.py --no-per-route --rate 100000 --period-ms 10 > gpurun_out/churn_100k.json 2>/dev/null
cp grout_amd/libgrout_hip.so /tmp/cur.so
cp build/ab/new.so grout_amd/libgrout_hip.so
python tools/fib_churn.py --no-per-route --rate 10000 --period-ms 10 > gpurun_out/churn_blocking.json 2>/dev/null || true
cp /tmp/cur.so grout_amd/libgrout_hip.so
