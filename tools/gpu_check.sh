#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel trace. Each GPU step has
# its own time limit; a crash, abort or timeout ends the script (no retries).
# A plain test failure (pytest exit 1) still lets the bench run.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

stop_if_fatal() { # $1 = exit status, $2 = step
	local s=$1
	if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then
		echo "FATAL: $2 exited $s, stopping" | tee -a $OUT/steps.log
		exit "$s"
	fi
	echo "$2 exit $s" | tee -a $OUT/steps.log
}

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -30 $OUT/pytest_gpu.log

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
stop_if_fatal $? smoke
cat $OUT/smoke.log

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
stop_if_fatal $? bench
cat $OUT/bench.json; tail -5 $OUT/bench.err

if [ -n "$PROFILE" ]; then
	timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
		python3 bench.py --no-cpu-baseline --no-host-path --steps 10 --warmup 3 > $OUT/prof_bench.json 2> $OUT/prof.err
	stop_if_fatal $? rocprof
fi
exit 0
