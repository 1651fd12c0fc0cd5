#!/bin/bash
# One gpurun call = a chain of named steps, each under its own time limit, chained so that a
# crash / abort / timeout ends the call (a plain test FAILURE, rc 1, lets later steps run).
#   bash scripts/gpu_run.sh <outdir> suite smoke bench iso prof ...
# Outputs land in gpurun_out/<outdir>/.
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$1; shift
mkdir -p "$O"
T="timeout -k 10"
PYT="python -u -m pytest -v --timeout 120 --timeout-method thread"
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for step in "$@"; do
  case $step in
    suite) $T 900 $PYT tests -m gpu > $O/suite.txt 2>&1 ;;
    suitex) $T 900 $PYT -x tests -m gpu > $O/suite.txt 2>&1 ;;
    tests:*) $T 600 $PYT -m gpu ${step#tests:} > $O/tests_$(basename ${step#tests:} .py).txt 2>&1 ;;
    smoke) $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 ;;
    bench) $T 600 python -u bench.py > $O/bench.json 2> $O/bench.err ;;
    benchgloo) $T 600 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err ;;
    iso) $T 300 python -u scripts/debug/stem_isolation.py > $O/stem_isolation.jsonl 2>&1 ;;
    det:*) a=${step#det:}; $T 300 python -u scripts/debug/determinism_probe.py --model ${a%%@*} --hw ${a##*@} >> $O/determinism.jsonl 2>&1 ;;
    probe:*) IFS=@ read -r m b sh reps opt <<< "${step#probe:}"
             $T 300 python -u scripts/overlap_probe.py --model $m --batch $b --shard ${sh:-0} --reps ${reps:-1} \
               --optimizer ${opt:-sgd} ${PROBE_ARGS:-} >> $O/overlap_probe.jsonl 2>> $O/overlap_probe.err ;;
    gossip:*) IFS=@ read -r m b opt dt <<< "${step#gossip:}"
             $T 400 python -u scripts/overlap_probe.py --gossip --model $m --batch $b --optimizer ${opt:-adam} \
               --grad-comm ${dt:-bf16} >> $O/gossip_probe.jsonl 2>> $O/gossip_probe.err ;;
    probetrace:*) IFS=@ read -r m b sh reps opt <<< "${step#probetrace:}"
             (cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
             $T 400 rocprofv3 --kernel-trace -d $O/probetrace_${m}_$sh -o run -- python -u scripts/overlap_probe.py \
               --model $m --batch $b --shard ${sh:-0} --reps ${reps:-1} --optimizer ${opt:-sgd} --rounds 1 --steps 5 --tail-steps 3 \
               > $O/probetrace_${m}_$sh.txt 2>&1) ;;
    phase:*) m=${step#phase:}; LDNN_CONV_XF=32 $T 300 python -u scripts/conv_phase_trace.py --model $m >> $O/phase_$m.jsonl 2>> $O/phase.err ;;
    mlpab) rc=0   # same-box A/B of MLP_AB_ENVS on the headline bench (MLP only), alternated 3x
           for r in 1 2 3; do for e in ${MLP_AB_ENVS:-X=0}; do
             echo "{\"rep\": $r, \"env\": \"$e\"}" >> $O/mlpab.jsonl
             env $e $T 200 python -u bench.py --no-configs >> $O/mlpab.jsonl 2>> $O/mlpab.err || { rc=$?; break 2; }
           done; done; (exit $rc) ;;
    gemmxf:*) $T 300 python -u scripts/gemm_q_xf.py --K ${step#gemmxf:} --variants ${XF_VARIANTS:-32,33,37,96,160} \
               >> $O/gemmxf.jsonl 2>> $O/gemmxf.err ;;
    script:*) f=${step#script:}; $T 300 python -u scripts/$f >> $O/${f%.py}.jsonl 2>> $O/${f%.py}.err ;;
    micro:*) m=${step#micro:}; rc=0
             for e in ${MICRO_ENVS:-X=0}; do
               echo "{\"env\": \"$e\"}" >> $O/micro_$m.jsonl
               env $e $T 300 python -u scripts/conv_micro.py --model $m --no-stock >> $O/micro_$m.jsonl 2>> $O/micro.err || { rc=$?; break; }
             done; (exit $rc) ;;
    ab:*) a=${step#ab:}; rm -f gpurun_out/ab_cnn.jsonl; $T 900 bash scripts/ab_cnn.sh "${a//,/ }" ${AB_ENVS:-X=0} >> $O/ab.txt 2>&1
          rc=$?; cat gpurun_out/ab_cnn.jsonl >> $O/ab_cnn.jsonl 2>/dev/null; (exit $rc) ;;
    microprof:*) m=${step#microprof:}; (cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
             $T 400 rocprofv3 --kernel-trace --stats -d $O/microprof_$m -o run -- \
             python -u scripts/conv_micro.py --model $m --no-stock --iters 20 > $O/microprof_$m.txt 2>&1) ;;
    micropmc:*) m=${step#micropmc:}; (cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
             timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
               SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/micropmc_$m -o run -- \
             python -u scripts/conv_micro.py --model $m --no-stock --iters 5 > $O/micropmc_$m.txt 2>&1) ;;
    cnn:*) a=${step#cnn:}; $T 300 python -u scripts/bench_cnn.py --model ${a%%@*} --batch ${a##*@} --graph --no-stock \
             >> $O/cnn.jsonl 2>> $O/cnn.err ;;
    prof:*) a=${step#prof:}; $T 400 rocprofv3 --kernel-trace --stats -d $O/prof_$a -o prof_${a%%@*}_${a##*@} -- \
             python -u scripts/bench_cnn.py --model ${a%%@*} --batch ${a##*@} --graph --no-stock --steps 20 --warmup 5 \
             > $O/prof_$a.txt 2>&1 ;;
    profmlp) $T 400 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o prof_mlp -- python -u bench.py --steps 20 --warmup 5 \
             --no-configs > $O/prof_mlp.txt 2>&1 ;;
    pmc:*) IFS=@ read -r tg m b <<< "${step#pmc:}"
           if [ "$m" = mlp3 ]; then $T 400 bash scripts/pmc_step.sh $tg python3 bench.py --steps 4 --warmup 3 --no-configs > $O/pmc_$tg.txt 2>&1
           else $T 400 bash scripts/pmc_step.sh $tg python3 scripts/bench_cnn.py --model $m --batch $b --steps 3 --warmup 2 --no-stock > $O/pmc_$tg.txt 2>&1; fi
           rc=$?; cp -f gpurun_out/pmc_$tg/table.txt $O/pmc_${tg}_table.txt 2>/dev/null; (exit $rc) ;;
    wsbench) $T 200 python -u scripts/bench_ws64.py >> $O/bench_ws64.jsonl 2>> $O/bench_ws64.err ;;
    wspmc) (cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
           timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
             SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/wspmc/p1 -o run -- \
             python3 scripts/bench_ws64.py --modes 0,1 --batches 256 > $O/wspmc_p1.log 2>&1 &&
           timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
             GRBM_GUI_ACTIVE --output-format csv -d $O/wspmc/p2 -o run -- \
             python3 scripts/bench_ws64.py --modes 0,1 --batches 256 > $O/wspmc_p2.log 2>&1) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" | tee -a $O/steps.txt
  if fatal $rc; then echo "fatal rc=$rc at $step: stopping"; exit $rc; fi
done
