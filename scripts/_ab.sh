cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
AB_TAG=new timeout -k 10 120 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1 || exit 1
OPOSE_LIB=alt_lib/base.so AB_TAG=base timeout -k 10 120 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1 || exit 1
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        r=json.loads(l); d[(r['layer'],r['tag'])].append(r['tf'])
for (layer,tag),v in sorted(d.items()): print(f"{layer:12s} {tag:6s} {' '.join(f'{x:6.1f}' for x in v)}")
PY
