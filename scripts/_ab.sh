cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
export AB_LAYERS=Mconv2-5,conv3_x,conv1_2
for v in cur abl1 abl2 abl3 abl8 abl11 abl16 abl32 cur; do
  if [ $v = cur ]; then L=pytorch-openpose_amd/lib/libopose.so; else L=alt_lib/$v.so; fi
  OPOSE_LIB=$L AB_TAG=$v timeout -k 10 60 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1 || exit 1
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        r=json.loads(l); d[r['layer']].append((r['tag'], r['tf']))
for k,v in d.items(): print(k, ' '.join(f'{t}:{x}' for t,x in v))
PY
