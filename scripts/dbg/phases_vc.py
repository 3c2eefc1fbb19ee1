"""Per-phase cycle stamps of the fused Decoder kernels (scripts/dbg/build_phases_vc.sh): mean over
the launches after the first 4 (workgroup 0), per wave, for tags dfwd / dbwd."""
import collections
import sys

runs = collections.defaultdict(list)   # (tag, wave) -> list of launches, each a list of cycles
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/phv.log"):
    p = l.split()
    if len(p) != 4 or p[0] not in ("dfwd", "dbwd"):
        continue
    tag, w, i, v = p[0], p[1], int(p[2]), int(p[3])
    if i == 1:
        runs[(tag, w)].append([])
    runs[(tag, w)][-1].append(v)
for tag in ("dfwd", "dbwd"):
    for w in ("w0", "w1", "w2", "w3"):
        L = runs[(tag, w)][4:]
        if not L:
            continue
        n = min(len(x) for x in L)
        m = [sum(x[k] for x in L) / len(L) for k in range(n)]
        print(tag, w, "launches", len(L), "total", int(sum(m)))
        print("  " + " ".join(f"{k + 1}:{int(v)}" for k, v in enumerate(m)))
