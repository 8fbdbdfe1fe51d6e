cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
export AB_LAYERS=Mconv1,conv3_x,conv4_2
for t in 128x256 256x128 128x256 256x128; do AB_TILE=$t AB_TAG=$t timeout -k 10 120 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1 || exit 1; done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        r=json.loads(l); d[r['layer']].append((r['tag'], r['tf']))
for k,v in d.items(): print(f"{k:12s}", ' '.join(f'{t}:{x}' for t,x in v))
PY
