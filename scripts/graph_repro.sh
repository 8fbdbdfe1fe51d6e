#!/bin/bash
# Run scripts/graph_fork_repro under /opt/rocm's HIP (7.2) and under torch's bundled HIP (7.0.2,
# the runtime libopose binds to when torch is imported first); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TL=$(python3 -c "import os, importlib.util as u; print(os.path.join(os.path.dirname(u.find_spec('torch').origin), 'lib'))")
# torch ships libamdhip64.so (SONAME libamdhip64.so.7): expose it under the name the binary needs
mkdir -p /tmp/hip70 && ln -sf "$TL/libamdhip64.so" /tmp/hip70/libamdhip64.so.7
TORCH_HIP="LD_LIBRARY_PATH=/tmp/hip70:$TL"
run() {  # tag, env, args...
    local tag=$1 envs=$2; shift 2
    env $envs timeout -k 10 120 ./scripts/graph_fork_repro "$@" > gpurun_out/gr_$tag.log 2>&1
    local rc=$?
    grep -m1 "^runtime" gpurun_out/gr_$tag.log
    grep "SIGNAL" gpurun_out/gr_$tag.log
    echo "$tag rc=$rc: $(tail -1 gpurun_out/gr_$tag.log)"
    return $rc
}
# the variants expected to pass first: a crash ends the call (nothing runs on the GPU after it)
case "${2:-all}" in
all)
    run rocm_stress "" stress ${1:-4000} &&
    run torch_fresh "$TORCH_HIP" fresh 200 &&
    run torch_reuse "$TORCH_HIP" reuse 200 &&
    run torch_stress "$TORCH_HIP" stress ${1:-4000} ;;
bisect)  # round 4's two conditions, now without libopose: no fork in captures / no exec destroyed
    run torch_stress_nofork "$TORCH_HIP STRESS_NOFORK=1" stress ${1:-4000} &&
    run torch_stress_leak "$TORCH_HIP STRESS_LEAK=1" stress ${1:-4000} &&
    run rocm_stress "" stress ${1:-4000} &&
    run torch_stress "$TORCH_HIP" stress ${1:-4000} ;;
esac
