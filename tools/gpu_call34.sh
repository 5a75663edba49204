#!/bin/bash
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python tools/pcie_probe.py > $OUT/pcie.jsonl 2> $OUT/pcie.err
s=$?; cat $OUT/pcie.jsonl; tail -2 $OUT/pcie.err; exit $s
