"""Per-call kernel time of the C2 replays (scripts/c2_replays.py under rocprofv3 --kernel-trace):
drops the 5 warm-up calls' kernels by keeping the last REPS x (kernels per call) dispatches."""
import csv, sys, collections
path, reps = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# kernels per call: the period of the name sequence at its end
n = len(rows)
for per in range(10, 400):
    if n >= per * (reps + 1) and names[n - per:] == names[n - 2 * per:n - per]:
        break
tail = rows[n - per * reps:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail) / reps / 1e3
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / reps / 1e3
print("kernels per call %d; per call: kernel time %.1f us, first start to last end %.1f us (incl. host gaps between calls)" % (per, busy, span))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in tail:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-70s %4d calls %8.1f us per call  %6.2f us mean" % (k[:70], c // reps, us / reps, us / c))
