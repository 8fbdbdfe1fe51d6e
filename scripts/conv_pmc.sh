#!/bin/bash
# Counter passes (rocprofv3 --pmc, one group per pass, no tracing domains) over the 7x7 conv
# kernel for a list of ablation variants; summary -> gpurun_out/convpmc/summary.txt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/convpmc
mkdir -p $OUT
i=0
for ab in ${ABLATES:-0 16}; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL" \
             "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
             "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum" "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -k 5 45 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python3 scripts/conv_probe.py $ab > $OUT/p$i.log 2>&1
    rc=$?
    echo "ab=$ab pass $i rc=$rc $(tail -1 $OUT/p$i.log)"
    case $rc in 124|137|139) exit $rc;; esac
  done
done
python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/convpmc/p*/**/*_counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "conv_igemm" in row["Kernel_Name"]:
            agg[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:40s} {sum(v) / len(v):18.6g}  (n={len(v)})")
PY
cat $OUT/summary.txt
