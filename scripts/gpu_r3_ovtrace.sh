#!/bin/bash
# kernel trace of the overlap probe (ResNet-18 b64): are the stand-in copies concurrent with the backward?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3/ovtrace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/ovtrace -o ov -- python3 scripts/overlap_probe.py --model resnet18 --batch 64 --steps 5 > gpurun_out/r3/ovtrace/probe.txt 2>&1 || { tail -20 gpurun_out/r3/ovtrace/probe.txt; exit 1; }
tail -2 gpurun_out/r3/ovtrace/probe.txt
find gpurun_out/r3/ovtrace -name "*.csv" | head
