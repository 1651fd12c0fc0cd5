#!/bin/bash
# PMC counter passes over a few CNN training steps (ldnn path): scripts/pmc_cnn.sh <model> <batch>
set -e
m=${1:-resnet18}; b=${2:-64}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmc_$m; mkdir -p $d
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $d/p$1_ -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 3 --warmup 2 --no-stock > $d/log 2>&1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $d/p1 -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 3 --warmup 2 --no-stock > $d/log1 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA --output-format csv -d $d/p2 -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 3 --warmup 2 --no-stock > $d/log2 2>&1
for k in "FwdA<128" "FwdA<256" "DgradA<128" "DgradA<256" "WgradA<128" "WgradA<64" "bn_reduce_kernel<false" "bn_apply"; do
  echo "== $k"; python3 scripts/pmc_summary.py $d "$k"
done > $d/summary.txt
cat $d/summary.txt
