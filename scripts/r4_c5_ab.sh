# Same-box A/B of one C5 scale network: alt_lib/pre_small.so = scripts/build_alt.sh 388af73 pre_small
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for r in 1; do
OPOSE_LIB=alt_lib/pre_small.so timeout -k 10 120 python scripts/c5_layers.py 3 > gpurun_out/c5l_pre_$r.log 2>&1 || { tail -3 gpurun_out/c5l_pre_$r.log; exit 1; }
timeout -k 10 120 python scripts/c5_layers.py 3 > gpurun_out/c5l_cur_$r.log 2>&1 || { tail -3 gpurun_out/c5l_cur_$r.log; exit 1; }
echo "pre: $(grep -v amdgpu gpurun_out/c5l_pre_$r.log | head -2 | tr '\n' ' ')"; echo "cur: $(grep -v amdgpu gpurun_out/c5l_cur_$r.log | head -2 | tr '\n' ' ')"
done
