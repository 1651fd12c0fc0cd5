set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5ovl; mkdir -p $O
for e in X=0 LDNN_RCCL_HIGH_PRIO=0 LDNN_DP_OPT_ORDER=forward; do
  echo "== $e" >> $O/t.txt
  env $e timeout -k 10 200 python -u -c "
from ldnn.parallel.overlap_probe import measure_overlap
import json
r = measure_overlap('lenet5', batch=1024, bucket_mb=0.05, reps=64, steps=20, blocks=8)
print(json.dumps({k: r[k] for k in ('single_ms','with_standin_ms','standin_alone_ms','segments') if k in r}))
" >> $O/t.txt 2>&1 || exit 3
done
