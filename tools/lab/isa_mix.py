"""Lab: VALU instruction mix of a kernel's loops in a device assembly file (hipcc --cuda-device-only -S).
usage: isa_mix.py FILE.s NAME_SUBSTRING [N_LOOPS]"""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
nloops = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lines = open(path).read().split("\n")
i = 0
while i < len(lines):
    m = re.match(r"^(_Z\w+):", lines[i])
    if not (m and pat in m.group(1)):
        i += 1
        continue
    name = m.group(1)
    j = i + 1
    while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
        j += 1
    body = lines[i + 1:j]
    labels = {}
    instrs = []  # (line index, op)
    for k, l in enumerate(body):
        t = l.strip()
        lm = re.match(r"^(\.LBB\w+):", t)
        if lm:
            labels[lm.group(1)] = k
            continue
        if not t or t.startswith((".", ";")):
            continue
        instrs.append((k, t.split()[0], t))
    loops = []
    for k, op, t in instrs:
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] < k:
                loops.append((labels[tgt], k))
    total = collections.Counter(op for _, op, _ in instrs)
    print(f"{name}: {sum(total.values())} instrs, {sum(v for o, v in total.items() if o.startswith('v_'))} VALU")
    for a, b in sorted(loops, key=lambda ab: -(ab[1] - ab[0]))[:nloops]:
        c = collections.Counter(op for k, op, _ in instrs if a <= k <= b)
        v = sum(n for o, n in c.items() if o.startswith("v_"))
        print(f"  loop lines {a}-{b}: {sum(c.values())} instrs, VALU {v}: " +
              ", ".join(f"{o} {n}" for o, n in c.most_common(14)))
    i = j
