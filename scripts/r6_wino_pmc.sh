#!/bin/bash
# PMC passes over a short serial bench (conv_wino_x6 against conv_win_x6's 3x3 layers)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1 BENCH_PIPELINE=0
OUT=gpurun_out/wprof; mkdir -p $OUT
ARGS="bench.py --steps 2 --warmup 1 --no-cpu --latency-iters 0 --host-steps 1"
for p in "pmc1:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "pmc2:SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "pmc5:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS"; do
  name=${p%%:*}; ctr=${p#*:}
  timeout -k 10 240 rocprofv3 --pmc $ctr -d $OUT/$name -o $name --output-format csv -- python3 $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -3 $OUT/$name.log; exit 1; }
done
python3 - <<'PY'
import glob, pandas as pd
rows=[]
for f in glob.glob("gpurun_out/wprof/pmc*/**/*counter_collection.csv", recursive=True):
    d=pd.read_csv(f); rows.append(d)
d=pd.concat(rows)
d=d[d.Kernel_Name.str.contains("conv_wino|conv_win_x6<128, 256, 3")]
d["k"]=d.Kernel_Name.str.slice(0,48)
t=d.groupby(["k","Counter_Name"]).Counter_Value.mean().unstack()
pd.set_option("display.width",250); pd.set_option("display.max_columns",30)
print(t.T.to_string())
PY
