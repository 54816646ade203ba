"""Development only: concurrency in a rocprofv3 kernel trace of bench.py's timed C2 steps
(python tools/lane_trace.py <kernel_trace.csv>): per queue, busy time over the last N steps'
window, and how much of the window has 0 / 1 / 2+ queues busy."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
       (re.search(r"(k_\w+|__amd\w+|\w+_kernel)", r["Kernel_Name"]) or [r["Kernel_Name"][:20]])[0])
      for r in rows]
# the window: from the 60th-last k_estep_chunk start to the last decode kernel end
# the timed steps' training passes run on the lanes' CU-masked streams (the queues that run
# nothing but k_estep_chunk); the window spans the last 30 of them
qs = {}
for s_, e_, q, n in ks:
    qs.setdefault(q, set()).add(n)
tq = {q for q, v in qs.items() if v == {"k_estep_chunk"}}
est = [k for k in ks if k[2] in tq]
t0, t1 = est[-30][0], est[-1][1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1 + 1]
print("window us", (t1 - t0) / 1e3, "kernels", len(win))
byq = {}
for s, e, q, n in win:
    byq.setdefault(q, []).append((s, e, n))
for q, v in sorted(byq.items()):
    busy = sum(e - s for s, e, _ in v)
    names = {}
    for s, e, n in v:
        names[n] = names.get(n, 0) + (e - s)
    print("queue", q, "busy us", round(busy / 1e3, 1), {k: round(x / 1e3, 1) for k, x in sorted(names.items(), key=lambda x: -x[1])[:6]})
ev = []
for s, e, q, n in win:
    ev.append((s, 1, q))
    ev.append((e, -1, q))
ev.sort()
act = {}
last = t0
hist = {}
for t, d, q in ev:
    nq = sum(1 for v in act.values() if v > 0)
    hist[nq] = hist.get(nq, 0) + (t - last)
    last = t
    act[q] = act.get(q, 0) + d
tot = sum(hist.values())
print("queues busy at once (share of window):", {k: round(v / tot, 3) for k, v in sorted(hist.items())})
