# Packed-FP32 A/B: screened-NMS self-checks under overlap and the bench line, for the shipped
# library (no packed FP32) and alt_lib/pk.so (compiler default).  Historical record of the round-2
# root-cause run: the screened NMS and its debug script have since been deleted, so
# this no longer runs as is; scripts/pipeline_stress.sh is the current pipelined-records check.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
bash scripts/gauss_debug.sh main || true
for tag in main pk main pk; do
  lib=pytorch-openpose_amd/lib/libopose.so; [ "$tag" != main ] && lib=alt_lib/$tag.so
  OPOSE_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/b_$tag.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$tag.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('$tag', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in s.items()})"
done
