"""Per-phase cycle stamps of a long-engine -DAVC_FZ_PHASES run (workgroup 0, wave 0, last launch
of each tag): prints every stamp delta in order, and the total."""
import collections
import sys

seq = collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/phl.log"):
    p = line.split()
    if len(p) == 4 and p[0] in ("lfwd", "lbwd") and p[1].startswith("w"):
        seq[(p[0], p[1])].append((int(p[2]), int(p[3])))
for tag in ("lfwd", "lbwd"):
    for w in ("w0", "w1", "w2", "w3"):
        runs = []
        for i, v in seq[(tag, w)]:
            if i == 1:
                runs.append([])
            if runs:
                runs[-1].append(v)
        if not runs:
            continue
        last = runs[-1]
        print(f"{tag} {w}: {len(runs)} launches, last: {len(last)} stamps, total {sum(last)} cycles")
        print("  " + " ".join(f"{k + 1}:{v}" for k, v in enumerate(last)))
