set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fullview6 or clustered_routes6 or mixed_v4_v6 or live_route6 or host_scoping" > gpurun_out/sc_tests.log 2>&1
for i in 1 2; do
 for sc in 0 1 2; do  # 2: table staged, never read
  timeout -k 10 240 python bench.py --workload fullview6 --tune v6_shortcut=$sc >> gpurun_out/sc_ab.jsonl 2>> gpurun_out/sc_ab.err
 done
done
