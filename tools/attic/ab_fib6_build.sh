#!/bin/bash
# SPDX-License-Identifier: BSD-3-Clause
# Measurement builds of the FIB6 compactions for tools/ab_libs.sh: the same
# kernel object, fib6.c with range groups and / or narrow wide groups off.
#   off: neither (round 2's trie); narrow: narrow wide groups only;
#   range: range groups only; new: both (the default build)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ab
for v in off narrow range new; do
	case $v in
	off) D="-DFIB6_NO_RANGE -DFIB6_NO_NARROW" ;;
	narrow) D="-DFIB6_NO_RANGE" ;;
	range) D="-DFIB6_NO_NARROW" ;;
	new) D="" ;;
	esac
	gcc -O3 -march=x86-64-v3 -fPIC -Wall $D -c -o build/ab/fib6_$v.o grout_amd/csrc/fib6.c
	/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/$v.so build/fwd4_ring.o build/gr_hip.o \
		build/gr_node.o build/fib4.o build/ab/fib6_$v.o
done
