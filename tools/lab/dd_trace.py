"""Lab: kernel-trace window of the last C cycles of a DD run: busy time (union of kernel intervals) and the
per-kernel time per cycle.  dd_trace.py TRACE_DIR CYCLES MARKER (MARKER: a kernel name substring once per cycle)."""
import sys
from collections import defaultdict
sys.path.insert(0, __file__.rsplit("/", 3)[0] + "/tools")
from trace_summary import load, short  # noqa: E402

path, C, marker = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = sorted(load(path), key=lambda r: r[2])
idx = [i for i, r in enumerate(rows) if marker in r[0]]
lo, hi = idx[-C - 1], idx[-1]
win = rows[lo + 1:hi + 1]
t0, t1 = rows[lo][3], win[-1][3]
busy, cur_s, cur_e = 0, None, None
for _, _, s, e in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"window {C} cycles: span {(t1 - t0) / C / 1e3:.1f} us/cycle, busy {busy / C / 1e3:.1f} us/cycle, "
      f"{len(win) / C:.1f} kernels/cycle")
acc = defaultdict(lambda: [0, 0])
for n, gx, s, e in win:
    k = (short(n), gx)
    acc[k][0] += e - s
    acc[k][1] += 1
for (n, gx), (t, c) in sorted(acc.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f"{t / C / 1e3:8.2f} us/cycle  {c / C:5.2f}/cycle  avg {t / c / 1e3:7.2f}  {gx:9d}  {n}")
