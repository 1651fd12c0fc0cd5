#!/bin/bash
# PMC tables (MFMA utilisation, LDS bank conflicts, L2 hit) of the final tree: headline step and both CNN steps.
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/pmc_step.sh mlp3_final python3 bench.py --steps 4 --warmup 3 > /dev/null 2>&1 || exit $?
bash scripts/pmc_step.sh rn64_final python3 scripts/bench_cnn.py --model resnet18 --batch 64 --steps 4 --warmup 3 --no-stock --graph > /dev/null 2>&1 || exit $?
bash scripts/pmc_step.sh ecnn64_final python3 scripts/bench_cnn.py --model enhanced_cnn --batch 64 --steps 4 --warmup 3 --no-stock --graph > /dev/null 2>&1 || exit $?
for t in mlp3_final rn64_final ecnn64_final; do head -8 gpurun_out/pmc_$t/table.txt | cut -c1-150; done
