#!/bin/bash
# HBM bytes of the bandwidth-bound step kernels: one counter pass per TCC group.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=gpurun_out/pmc_membound
mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- python3 scripts/prof_membound.py > $o/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/p1 -o run -- python3 scripts/prof_membound.py > $o/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/p2 -o run -- python3 scripts/prof_membound.py > $o/p2.log 2>&1
