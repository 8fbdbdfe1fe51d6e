# Pipelined-records stress: mismatch counts for the current library and any alt_lib/*.so builds
# named in LIBS (older commits / single-change variants).  Found the limb_greedy shared-counter
# race (round 2): 2-3 subset mismatches per 840 frames before the fix.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TRIALS=${TRIALS:-40}
for lib in ${LIBS:-head head head}; do
  if [ $lib = head ]; then unset OPOSE_LIB; else export OPOSE_LIB=alt_lib/$lib.so; fi
  timeout -k 10 300 python -u scripts/pipeline_stress.py 2>&1 | grep "lib=" || exit 1
done
