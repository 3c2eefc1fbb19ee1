"""Print the per-phase cycle stamps of a -DAVC_FZ_PHASES run (wave 0, last launch)."""
import collections
import sys

lines = [l.split() for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ph.log") if l.startswith(("fwd", "bwd"))]
seq = collections.defaultdict(list)
for tag, w, i, v in lines:
    seq[(tag, w)].append((int(i), int(v)))
for tag in ("fwd", "bwd"):
    L = []
    for i, v in seq[(tag, "w0")]:
        if i == 1:
            L.append([])
        L[-1].append(v)
    if not L:
        continue
    last = L[-2] if len(L) > 1 else L[-1]
    print(tag, "total", sum(last))
    print("  " + " ".join(f"{k + 1}:{v}" for k, v in enumerate(last)))
