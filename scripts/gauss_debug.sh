# Screened Gaussian NMS under pipelined overlap (scripts/pipeline_check.py) with OPOSE_GAUSS_DEBUG:
# the float64 kernel runs after it into shadow lists and every difference is printed from the
# device.  Args: library tags ("main" = the built library, else alt_lib/<tag>.so).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for tag in "${@:-main}"; do
  lib=pytorch-openpose_amd/lib/libopose.so; [ "$tag" != main ] && lib=alt_lib/$tag.so
  L=gpurun_out/gdbg_$tag.log
  OPOSE_LIB=$lib OPOSE_GAUSS_SCREEN=1 OPOSE_GAUSS_DEBUG=1 timeout -k 10 300 python -u scripts/pipeline_check.py > $L 2>&1 || exit 1
  echo "$tag: frames differing from the host path $(grep -c ' frame ' $L), peaks missing vs float64 kernel $(grep -c 'GAUSSDBG.*missing' $L), extra $(grep -c 'GAUSSDBG.*extra' $L)"
done
