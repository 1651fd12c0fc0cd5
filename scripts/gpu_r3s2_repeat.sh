#!/bin/bash
# headline bench repeated on one box (run-to-run spread), default K/W and a longer run
set -o pipefail
O=gpurun_out/r3s2repeat
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-configs > $O/b$i.txt 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b$i.txt').read().strip().splitlines()[-1]); print('run $i', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u bench.py --no-configs --steps 300 --warmup 20 > $O/long.txt 2> $O/long.err || { tail -20 $O/long.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/long.txt').read().strip().splitlines()[-1]); print('300 steps', d['ms_per_step'], d['value'])"
