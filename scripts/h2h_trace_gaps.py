"""Per-step network start gaps from a rocprofv3 --kernel-trace --memory-copy-trace of scripts/h2h_ab.py:
for every preprocess_u8 launch, the idle time on its queue since the previous network's last kernel,
and how long after the latest assemble_people (the previous post-processing's end) it started.
A step whose network starts right after a post ends, with a gap, was held back behind that post.

    python scripts/h2h_trace_gaps.py gpurun_out/h2h_trace/run
"""
import sys

import pandas as pd


def main(prefix):
    k = pd.read_csv(prefix + "_kernel_trace.csv")
    m = pd.read_csv(prefix + "_memory_copy_trace.csv")
    t0 = min(k.Start_Timestamp.min(), m.Start_Timestamp.min())
    for d in (k, m):
        d["s"] = (d.Start_Timestamp - t0) / 1e6
        d["e"] = (d.End_Timestamp - t0) / 1e6
    pre = k[k.Kernel_Name.str.contains("preprocess_u8")]
    netq = pre.Queue_Id.mode()[0]
    q = k[k.Queue_Id == netq].sort_values("s").reset_index(drop=True)
    asm = k[k.Kernel_Name.str.contains("assemble_people")]
    print("queues: %s; network queue %d" % (dict(k.groupby("Queue_Id").size()), netq))
    print("copies (ms): %s" % m.assign(d=m.e - m.s).groupby(["Direction", "Stream_Id"]).d.agg(["count", "mean"]).to_dict())
    held = 0
    for idx in q.index[q.Kernel_Name.str.contains("preprocess_u8")]:
        if idx == 0:
            continue
        gap = q.s[idx] - q.e[idx - 1]
        a = asm[asm.e <= q.s[idx] + 1e-3]
        after_post = q.s[idx] - a.e.max() if len(a) else float("nan")
        flag = gap > 0.1 and after_post < 0.1
        held += flag
        print("network at %10.3f ms  gap %7.3f ms  %7.3f ms after the last post%s"
              % (q.s[idx], gap, after_post, "  <- held behind the post" if flag else ""))
    print("held steps:", held)


if __name__ == "__main__":
    main(sys.argv[1])
