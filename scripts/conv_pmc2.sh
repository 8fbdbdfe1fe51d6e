#!/bin/bash
# counters for conv_probe2 variants: "<env> <ablate>" pairs in VARIANTS
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/convpmc2
mkdir -p $OUT
i=0
for v in "1 0" "0 0" "0 1" "0 2"; do
  set -- $v
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"; do
    i=$((i + 1))
    OPOSE_CONV_WINDOW=$1 timeout -k 5 60 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python3 scripts/conv_probe2.py $2 > $OUT/p$i.log 2>&1
    rc=$?
    echo "v=$v pass $i rc=$rc $(grep win= $OUT/p$i.log)"
    case $rc in 124|137|139) exit $rc;; esac
  done
done
python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/convpmc2/p*/**/*_counter_collection.csv", recursive=True):
    n = int(re.search(r"/p(\d+)/", f).group(1))
    var = (n - 1) // 4
    for row in csv.DictReader(open(f)):
        if "conv_" in row["Kernel_Name"] and "fixup" not in row["Kernel_Name"]:
            agg[(var, row["Kernel_Name"][:60])][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.6g}")
PY
cat $OUT/summary.txt
