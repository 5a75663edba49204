#!/bin/bash
# SPDX-License-Identifier: BSD-3-Clause
#
# One GPU session through gpurun: a list of steps, each under its own time
# limit, stopping at the first crash, abort, time limit or failure (no
# retries). Outputs land in gpurun_out/ (merged back by gpurun).
#
#   tools/gpu_session.sh STEP [STEP ...]
#
# Steps:
#   tests[=K]         pytest -m gpu (-k K)               -> pytest_gpu.log
#   smoke             __graft_entry__.smoke()            -> smoke.log
#   bench[:TAG][=A]   python bench.py A                  -> bench[_TAG].json
#   prof[:TAG][=A]    rocprofv3 --kernel-trace --stats of bench.py A -> prof[_TAG]/
#   pmc:TAG=SET[@A]   rocprofv3 --pmc SET (space separated counters, one pass)
#                     of tools/pmc_run.py A              -> pmc_TAG/
#                     (PMC_TIMEOUT seconds, default 120)
#   run:TAG=CMD       any command (a tools/ script)      -> run_TAG.log
#
# e.g. gpurun -- 'bash tools/gpu_session.sh tests smoke bench prof="--steps 20 --warmup 5 --no-cpu-baseline --no-host-path"'
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

fatal() { # $1 = exit status, $2 = step
	echo "$2 exit $1" | tee -a $OUT/steps.log
	[ "$1" -eq 0 ] || exit "$1"
}

for step in "$@"; do
	kind=${step%%=*}
	arg=""
	[ "$kind" != "$step" ] && arg=${step#*=}
	tag=""
	case "$kind" in *:*) tag=${kind#*:}; kind=${kind%%:*} ;; esac
	sfx=${tag:+_$tag}
	case "$kind" in
	tests)
		timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
			-p no:cacheprovider ${arg:+-k "$arg"} > $OUT/pytest_gpu$sfx.log 2>&1
		s=$?
		tail -3 $OUT/pytest_gpu$sfx.log
		fatal $s "tests$sfx"
		;;
	smoke)
		timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
		s=$?
		tail -2 $OUT/smoke.log
		fatal $s smoke
		;;
	bench)
		timeout -k 10 600 python bench.py $arg > $OUT/bench$sfx.json 2> $OUT/bench$sfx.err
		s=$?
		cat $OUT/bench$sfx.json
		tail -3 $OUT/bench$sfx.err
		fatal $s "bench$sfx"
		;;
	prof)
		rm -rf $OUT/prof$sfx
		timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$sfx -o run -- \
			python3 bench.py $arg > $OUT/prof$sfx.json 2> $OUT/prof$sfx.err
		s=$?
		cat $OUT/prof$sfx.json
		fatal $s "prof$sfx"
		;;
	pmc)
		set_=${arg%%@*}
		args=""
		[ "$set_" != "$arg" ] && args=${arg#*@}
		rm -rf $OUT/pmc$sfx
		timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $set_ --output-format csv -d $OUT/pmc$sfx -o run -- \
			python3 tools/pmc_run.py $args > $OUT/pmc$sfx.log 2>&1
		fatal $? "pmc$sfx"
		;;
	run)
		timeout -k 10 600 $arg > $OUT/run$sfx.log 2>&1
		s=$?
		tail -20 $OUT/run$sfx.log
		fatal $s "run$sfx"
		;;
	*)
		echo "unknown step $step" >&2
		exit 2
		;;
	esac
done
exit 0
