# rocprofv3 kernel stats of the C2 single-frame path (scripts/c2_profile.py: graph replays + a profiled pass)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c2prof && export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o c2 --output-format csv -- python3 scripts/${PROFILE_SCRIPT:-c2_profile.py} > gpurun_out/c2prof/log 2>&1; echo rc=$?
