"""Benchmark: defended utterances/s of the AdaIN-VC embedding attack
(n_iters=1500, eps=0.1) on MI355X — BASELINE.json `metric`, configs[1] workload
(B=256 utterances of 80x128 normalized mel per GPU, bf16 MFMA operands with fp32
accumulation / Adam state; the fp32 path is timed too and reported beside it).
--attack e2e / fb measure configs[2] / [3] (end-to-end and feedback attacks); --attack pm
measures configs[4] (VSMask PredictiveModel forward, windows/s of [B,1,80,100]);
--attack mel2wav measures the back end after the attack: denormalize +
mel2wav (inverse dB, inv_mel_matrix, 100 Griffin-Lim iterations, de-emphasis) of B defended
80x128 mels per GPU, vocoded utts/s.

One "step" = one complete 1500-iteration attack over the rank's batch
(inputs already resident in HBM).  N>1: one process per GPU, each rank attacks its
own contiguous shard of the global batch (no data-path collective; scaling "weak"),
barrier + max-over-ranks timing.  Under torchrun the ranks come from the environment;
`python bench.py --gpus N` without it launches the N rank processes itself (and fails
loudly when fewer than N GPUs are visible -- never a silent 1-GPU run).  --dry-run
exercises that launcher, the rendezvous (gloo), sharding, timing and the JSON line on
the CPU without computing an attack (the multi-rank CPU test drives it).

Also reported:
  roofline      dominant kernel's algorithmic FLOP / its average launch time
                (HIP events on libavc's stream, a separate profiled pass after
                the timed region) vs the gfx950 dense peak for the dtype.
  cpu_baseline  the reference loop on the host cores (oracle/torch_cpu.py: the
                reference's own ATen arithmetic, bitwise-pinned), rank 0 at N=1,
                on a bounded sample scaled to utts/s.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
# Committed tile-variant choices for this workload (libavc's autotune cache, written by an
# unprofiled tune run on an MI355X): bench, rocprofv3 runs and profiles/ then agree on the
# kernels launched.  Shapes missing from the file are tuned at first use.
os.environ.setdefault("AVC_TUNE_FILE", os.path.join(ROOT, "profiles", "tune_gfx950.txt"))
sys.path.insert(0, os.path.join(ROOT, "attack-vc_amd"))
sys.path.insert(0, ROOT)

FULL_CFG = {
    "SpeakerEncoder": dict(c_in=80, c_h=128, c_out=128, kernel_size=5, bank_size=8, bank_scale=1, c_bank=128,
                           n_conv_blocks=6, n_dense_blocks=6, subsample=[1, 2, 1, 2, 1, 2], act="relu",
                           dropout_rate=0.0),
    "ContentEncoder": dict(c_in=80, c_h=128, c_out=128, kernel_size=5, bank_size=8, bank_scale=1, c_bank=128,
                           n_conv_blocks=6, subsample=[1, 2, 1, 2, 1, 2], act="relu", dropout_rate=0.0),
    "Decoder": dict(c_in=128, c_cond=128, c_h=128, c_out=80, kernel_size=5, n_conv_blocks=6,
                    upsample=[2, 1, 2, 1, 2, 1], act="relu", sn=False, dropout_rate=0.0),
}
# FLOP per utterance-iteration (forward + input-gradient, ContentEncoder
# hoisted out of the loop for e2e / fb)
FLOP_PER_UTT_ITER = {"emb": 518_848_512, "e2e": 780_468_224, "fb": 1_299_316_736}
FLOP_PER_WINDOW = 204_457_536      # PredictiveModel forward per [1,80,100] window
# assumed AdaIN-VC config.yaml `preprocess` section (not in the container)
PREPROCESS = dict(sample_rate=16000, preemph=0.97, n_fft=2048, hop_length=300, win_length=1200, n_mels=80,
                  ref_db=20, max_db=100, top_db=15)
GL_ITERS = 100    # data_utils.py:172 (griffin_lim n_iter default)
HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md
PROF_ITERS = 10   # iterations of the HIP-event profiled pass (roofline)
KTIME_ITERS = 500  # graph-replayed iterations of the in-graph kernel timing pass (avc_ktime; ~0.1 s)
PEAK = {"fp32": (157.3, "TFLOP/s"), "bf16": (2500.0, "TFLOP/s")}   # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--n-iters", type=int, default=1500)
    ap.add_argument("--eps", type=float, default=0.1)
    ap.add_argument("--attack", default="emb", choices=["emb", "e2e", "fb", "pm", "mel2wav"])
    ap.add_argument("--precision", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--no-fp32-compare", action="store_true", help="skip the fp32 comparison step")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=12,
                    help="CPU baseline (ii): concurrent 1-thread processes (the GPU box's CPU share is 16; "
                         "its process guard allows 16 processes with the GPU open, this one included)")
    ap.add_argument("--cpu-worker", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--lengths", default=None, metavar="MIN:MAX",
                    help="emb attack over a seeded uniform mix of utterance lengths in [MIN, MAX] frames (real data: "
                         "every utterance its own length), one ragged batch per GPU (attack_many(ragged=True))")
    ap.add_argument("--bucketed", action="store_true",
                    help="--lengths: per-length buckets (attack_many's default) instead of the ragged batch, for comparison")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: launcher + gloo rendezvous + sharding + timing, no attack computed")
    return ap.parse_args()


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpu_count(nodes=KFD_NODES, dev_dir="/dev/dri") -> int:
    """GPUs this process can open, counted WITHOUT initialising HIP (launch_ranks must not: a process
    that has initialised the GPU may not fork the rank processes): the KFD topology nodes with a non-zero
    gpu_id whose DRM render node exists and is accessible, narrowed by ROCR_VISIBLE_DEVICES /
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as the runtime applies them.  Never calls into torch.cuda
    (torch's device_count falls back to hipGetDeviceCount when amdsmi is unavailable)."""
    n = 0
    try:
        names = sorted(os.listdir(nodes))
    except OSError:
        names = []
    for d in names:
        try:
            with open(os.path.join(nodes, d, "properties")) as fh:
                props = dict(ln.split(None, 1) for ln in fh.read().splitlines() if len(ln.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("gpu_id", "0").strip() or 0) == 0:
            continue                      # a CPU node
        minor = props.get("drm_render_minor", "").strip()
        if minor and not os.access(os.path.join(dev_dir, f"renderD{minor}"), os.R_OK | os.W_OK):
            continue                      # listed by the host's topology, not passed to this container
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(a) -> int:
    """--gpus N without torchrun: start N rank processes of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set like torchrun, 127.0.0.1 rendezvous) and return the worst exit
    code.  Nothing in this process touches the GPU: the count comes from sysfs (visible_gpu_count)."""
    import socket
    import subprocess
    if not a.dry_run:
        n = visible_gpu_count()
        if n < a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} requested but only {n} GPU(s) are visible; "
                             f"refusing to report a {n}-GPU number as {a.gpus}")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll: the first rank to fail ends the others (they would otherwise wait in the rendezvous or
    # a barrier until gloo's 30-minute timeout)
    codes = [None] * len(procs)
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(0.2)
    return max(codes, key=abs)


def main_dry_run(a):
    """The multi-rank path of main() on the CPU: gloo rendezvous, the rank's contiguous shard,
    barrier-bracketed timing, max over ranks, one JSON line from rank 0.  The "step" only
    touches the shard (no attack): this checks the orchestration, not the kernels."""
    import torch.distributed as dist_mod
    import shard
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        dist = dist_mod
        dist.init_process_group("gloo")
    total = a.batch * world
    sl = shard.shard_slice(total, rank, world)
    vc = torch.randn(total, 80, a.frames, generator=torch.Generator().manual_seed(1))[sl]
    for _ in range(a.warmup):
        vc.sum()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = vc.double().sum()
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, None)
    sizes = torch.tensor([sl.stop - sl.start], dtype=torch.int64)
    if dist:
        allz = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allz, sizes)
        sizes = torch.cat(allz)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "shard_sizes": [int(x) for x in sizes], "global_batch": total,
                          "value": round(total * a.steps / max(elapsed, 1e-9), 3), "checksum": float(s)}), flush=True)
    if dist:
        dist.destroy_process_group()


def _cpu_sample(model_sd, kind, budget_s, threads):
    """Time the reference loop (B=1, 80x128) for about budget_s seconds; returns
    (iterations timed, seconds per iteration)."""
    from oracle import torch_cpu
    torch.set_num_threads(threads)
    sd = model_sd
    g = torch.Generator().manual_seed(1)
    vc, at = torch.randn(1, 80, 128, generator=g), torch.randn(1, 80, 128, generator=g)
    p0 = torch.randn(1, 80, 128, generator=torch.Generator().manual_seed(123))
    src = torch.randn(1, 80, 128, generator=g)

    def run(n, hook=None):
        if kind == "emb":
            return torch_cpu.emb_attack(sd, FULL_CFG, vc, at, 0.1, n, p0, iter_hook=hook)
        return torch_cpu.vc_attack(kind, sd, FULL_CFG, src, vc, at, 0.1, n, p0, iter_hook=hook)

    run(3)                                                              # warm-up
    stamps = []
    t0 = time.perf_counter()

    def hook(it):
        stamps.append(time.perf_counter())
        if stamps[-1] - t0 > budget_s:
            raise StopIteration

    try:
        run(1500, hook)
    except StopIteration:
        pass
    return len(stamps), (stamps[-1] - t0) / len(stamps)


def cpu_worker(a):
    """--cpu-worker SECONDS: one 1-thread process of CPU baseline (ii); prints its sample."""
    import models
    torch.manual_seed(0)
    model = models.AdaInVC(FULL_CFG)
    n, per_iter = _cpu_sample({k: v.detach().cpu() for k, v in model.state_dict().items()}, a.attack, a.cpu_worker, 1)
    print(json.dumps({"iters": n, "per_iter": per_iter}), flush=True)


def cpu_baseline_throughput(kind, budget_s, procs):
    """BASELINE.md CPU baseline (ii): `procs` concurrent 1-thread processes, B=1 each (the
    throughput a CPU box gets from the reference), aggregated utts/s.  Child processes of
    this script (--cpu-worker), started with subprocess."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="",
               CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.abspath(__file__), "--attack", kind, "--cpu-worker", str(budget_s)]
    ps = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env)
          for _ in range(procs)]
    per = []
    for p in ps:
        out, _ = p.communicate(timeout=budget_s * 4 + 180)
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if p.returncode == 0 and lines:
            per.append(json.loads(lines[-1])["per_iter"])
    if not per:
        return None
    agg = sum(1.0 / (t * 1500) for t in per)
    return {"value": round(agg, 4), "unit": "utts/s", "cores": len(per), "kind": "port",
            "sample": f"{len(per)} concurrent 1-thread processes, B=1 {kind}_attack 80x128 each, ~{budget_s:.0f} s "
                      f"of iterations timed per process ({1e3 * min(per):.1f}-{1e3 * max(per):.1f} ms/iter), "
                      f"scaled x1500 and summed"}


def cpu_baseline(model, budget_s, kind="emb", procs=16):
    """Reference attack loop on the host: (i) as shipped -- one process, B=1, all host threads
    used by ATen -- and (ii) throughput -- `procs` concurrent 1-thread processes."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n, per_iter = _cpu_sample({k: v.detach().cpu() for k, v in model.state_dict().items()}, kind, budget_s, threads)
    out = {"value": 1.0 / (per_iter * 1500), "unit": "utts/s", "cores": threads, "kind": "port",
           "sample": f"B=1 {kind}_attack 80x128, {n} of 1500 iterations timed ({per_iter*1e3:.2f} ms/iter), "
                     f"scaled x1500; oracle/torch_cpu.py (reference ATen arithmetic incl. weight grads)"}
    if procs > 0:
        out["throughput"] = cpu_baseline_throughput(kind, min(budget_s, 15.0), procs)
    return out


def cpu_baseline_pm(budget_s, sd):
    """Reference PredictiveModel eval forward (ATen CPU, all host threads), B=1 windows."""
    from oracle import torch_cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    x = torch.randn(1, 1, 80, 100, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        torch_cpu.pm_forward(sd, x)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            torch_cpu.pm_forward(sd, x)
            n += 1
    dt = (time.perf_counter() - t0) / n
    return {"value": round(1.0 / dt, 2), "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"{n} B=1 forwards of a [1,1,80,100] window ({dt * 1e3:.2f} ms each); oracle/torch_cpu.pm_forward "
                      f"(reference ATen arithmetic)"}


def main_pm(a):
    """configs[4]: PredictiveModel forward over B windows per GPU (step = one batched forward)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max only: no RCCL in the process
    import avc_native
    import predictive_model
    import shard
    torch.manual_seed(0)
    m = predictive_model.PredictiveModel().eval()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    md = m.to(dev)
    B = a.batch
    total = B * world
    x_all = torch.randn(total, 1, 80, 100, generator=torch.Generator().manual_seed(1))
    x = x_all[shard.shard_slice(total, rank, world)].contiguous().to(dev)
    steps = max(a.steps, 20)                 # a step is ~ms: time at least 20 of them
    for _ in range(max(a.warmup, 3)):
        md(x)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        y = md(x)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, None)
    assert torch.isfinite(y).all()
    cpu = cpu_baseline_pm(min(a.cpu_seconds, 10.0), sd) if rank == 0 and world == 1 and not a.no_cpu_baseline else None
    if rank == 0:
        value = total * steps / elapsed
        achieved = FLOP_PER_WINDOW * value / world / 1e12
        # HBM bytes of one forward from the committed PMC passes (scripts/r03_pm_prof.sh ->
        # profiles/r04_pm_summary.md), summed over its kernels -- measured at one batch size, so reported
        # only when this run's per-GPU batch is that one (null otherwise)
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        pm_rec = json.load(open(tpath)).get("pm", {}) if os.path.exists(tpath) else {}
        pm_traffic = pm_rec.get("forward") if pm_rec.get("batch") == B else None
        print(json.dumps({
            "metric": "PredictiveModel windows/sec ([B,1,80,100] eval forward); 1/2/4/8 MI355X", "value": round(value, 1),
            "unit": "windows/s", "n_gpus": world, "steps": steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"PredictiveModel forward B={B}/GPU (BASELINE configs[4]; random init seed 0)",
                       "batch_per_gpu": B, "parallelism": f"dp{world} (independent window shards, no collective)"},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK["fp32"][0], "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK["fp32"][0], 4), "traffic": pm_traffic,
                         "kernel": "PredictiveModel forward (pm_cin1, pm_mfma x 10, pm_cout1 + split-K pm_reduce)"},
            "cpu_baseline": cpu, "flop_per_window": FLOP_PER_WINDOW,
            "libavc": avc_native.lib().avc_version().decode()}), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_mel2wav(budget_s, mel):
    """The reference's mel2wav (numpy float64 restatement of data_utils.py:121-197 with
    librosa 0.8 semantics, oracle/mel_dsp.py) on one utterance, host threads as numpy uses them."""
    from oracle import mel_dsp
    pre = {k: v for k, v in PREPROCESS.items() if k != "top_db"}
    t0 = time.perf_counter()
    n = 0
    while True:
        mel_dsp.mel2wav(mel, **pre, n_iter=GL_ITERS)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = (time.perf_counter() - t0) / n
    return {"value": round(1.0 / dt, 4), "unit": "utts/s", "cores": 1, "kind": "port",
            "sample": f"{n} single-utterance mel2wav calls (80x{mel.shape[0]} mel, {GL_ITERS} Griffin-Lim iterations, "
                      f"{dt:.2f} s each); oracle/mel_dsp.py (numpy pocketfft, float64, one thread)"}


def main_mel2wav(a):
    """Back end: B defended mels per GPU -> waveforms (step = one batched mel2wav)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max only: no RCCL in the process
    import avc_native
    import data_utils
    import shard
    B, T = a.batch, a.frames
    total = B * world
    g = torch.Generator().manual_seed(1)
    # normalized mels ~ N(0,1) (data_utils.py:35-47) with per-bin statistics of a dB-scaled
    # spectrogram in [0, 1]
    mean = torch.linspace(0.35, 0.55, 80, dtype=torch.float64)
    std = torch.linspace(0.12, 0.2, 80, dtype=torch.float64)
    mel_all = torch.randn(total, 80, T, generator=g)
    mel = mel_all[shard.shard_slice(total, rank, world)].contiguous().to(dev)
    attr = {"mean": mean.numpy(), "std": std.numpy()}
    d = data_utils.dsp_for(PREPROCESS, dev)

    def step():
        return d.mel2wav(mel, attr["mean"], attr["std"], True, GL_ITERS)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, None)
    assert torch.isfinite(out).all()
    roof = None
    if not a.no_roofline:
        d.set_profiling(True)
        step()
        stats = d.profile()
        d.set_profiling(False)
        N, hop = PREPROCESS["n_fft"], PREPROCESS["hop_length"]
        F = N // 2 + 1
        Tf = T
        # algorithmic HBM bytes per frame: dsp_gl_frames reads the target magnitude (F) and
        # the signal's new samples (hop), writes the windowed frame (N); dsp_ola reads the
        # frames (N) and writes the signal (hop)
        per_frame = {"dsp_gl_frames": (F + hop + N) * 4, "dsp_ola": (N + hop) * 4}
        name = "dsp_gl_frames"
        n, ms = stats[name]
        avg = ms / n
        achieved = per_frame[name] * B * Tf / (avg * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK, 4), "traffic": None, "kernel": name,
                "avg_launch_ms": round(avg, 4), "bytes_per_launch": per_frame[name] * B * Tf,
                "per_kernel": {k: {"launches": v[0], "avg_ms": round(v[1] / v[0], 4)} for k, v in stats.items()}}
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tpath):
            tr = json.load(open(tpath)).get("mel2wav", {}).get(name)
            if tr is not None:
                roof["traffic"] = tr
    # front end on the same shapes: B trimmed waveforms of hop * (T - 1) samples -> normalized
    # [B, 80, T] mels (file2mel after load / trim + normalize, one dsp_wav2mel launch)
    wav = out.contiguous()
    for _ in range(3):
        d.wav2mel(wav, attr["mean"], attr["std"], True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        mel_fe = d.wav2mel(wav, attr["mean"], attr["std"], True)
    e1.record()
    torch.cuda.synchronize()
    fe_ms = e0.elapsed_time(e1) / 20
    assert mel_fe.shape == (B, 80, T) and torch.isfinite(mel_fe).all()
    fe_bytes = B * (wav.shape[1] + 80 * T) * 4          # algorithmic: read the waveform, write the mel
    front = {"kernel": "dsp_wav2mel", "utts_per_s": round(B / (fe_ms * 1e-3), 1), "avg_launch_ms": round(fe_ms, 4),
             "bytes_per_launch": fe_bytes, "hbm_frac": round(fe_bytes / (fe_ms * 1e-3) / 1e9 / HBM_PEAK, 4)}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import numpy as np
        m0 = (mel[0].T.double().cpu().numpy() * attr["std"] + attr["mean"]).astype(np.float32)
        cpu = cpu_baseline_mel2wav(min(a.cpu_seconds, 20.0), m0)
    if rank == 0:
        print(json.dumps({
            "metric": f"vocoded utts/sec (denormalize + mel2wav, {GL_ITERS} Griffin-Lim iterations, 80x{T} mel); "
                      "1/2/4/8 MI355X", "value": round(total * a.steps / elapsed, 2), "unit": "utts/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"mel2wav B={B}/GPU, 80x{T} normalized mels, preprocess {PREPROCESS} "
                                   f"(assumed AdaIN-VC config)", "batch_per_gpu": B, "frames": T,
                       "parallelism": f"dp{world} (independent utterance shards, no collective)"},
            "roofline": roof, "cpu_baseline": cpu, "front_end_wav2mel": front,
            "libavc": avc_native.lib().avc_version().decode()}), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_lengths(sd, lens, budget_s, threads, mean_T):
    """The reference loop (oracle/torch_cpu.py, B = 1) over utterances of the mix, for about budget_s
    seconds: frame-iterations per second, scaled to utts/s of the mix (x 1500 iterations, mean length)."""
    from oracle import torch_cpu
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(5)
    done_fi, t_used, used = 0, 0.0, []
    for T in lens:
        vc, at, p0 = (torch.randn(1, 80, T, generator=g) for _ in range(3))
        torch_cpu.emb_attack(sd, FULL_CFG, vc, at, 0.1, 1, p0)           # warm-up of this shape
        stamps = []
        t0 = time.perf_counter()

        def hook(it):
            stamps.append(time.perf_counter())
            if stamps[-1] - t0 > budget_s / 4:
                raise StopIteration
        try:
            torch_cpu.emb_attack(sd, FULL_CFG, vc, at, 0.1, 1500, p0, iter_hook=hook)
        except StopIteration:
            pass
        done_fi += T * len(stamps)
        t_used += stamps[-1] - t0
        used.append(T)
        if t_used > budget_s:
            break
    rate = done_fi / t_used                       # frame-iterations per second
    return {"value": round(rate / (mean_T * 1500), 5), "unit": "utts/s", "cores": threads, "kind": "port",
            "frames_per_s": round(rate / 1500, 2),
            "sample": f"B=1 emb_attack of {len(used)} utterances of the mix ({used} frames), {done_fi} "
                      f"frame-iterations in {t_used:.1f} s, scaled to the mix's mean length {mean_T:.1f} x 1500 "
                      f"iterations; oracle/torch_cpu.py (reference ATen arithmetic)"}


def main_lengths(a):
    """Real-data lengths: B utterances per GPU, lengths uniform in [MIN, MAX] (seeded), adv_tgt of their own
    seeded lengths; step = attack_many(ragged=True) -- the adv_tgt embeddings per length plus one ragged
    1500-iteration attack over the rank's utterances (every pass one launch over all lengths)."""
    lo, hi = (int(v) for v in a.lengths.split(":"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max only: no RCCL in the process
    import avc_native
    import batching
    import models
    import shard
    torch.manual_seed(0)
    model = models.AdaInVC(FULL_CFG)
    model_dev = model.to(dev)
    B = a.batch
    total = B * world
    g = torch.Generator().manual_seed(2)
    lens_all = torch.randint(lo, hi + 1, (total,), generator=g).tolist()
    alens_all = torch.randint(lo, hi + 1, (total,), generator=g).tolist()
    sl = shard.shard_slice(total, rank, world)
    lens, alens = lens_all[sl], alens_all[sl]
    gi = torch.Generator().manual_seed(3 + rank)
    vc = [torch.randn(80, t, generator=gi).to(dev) for t in lens]
    at = [torch.randn(80, t, generator=gi).to(dev) for t in alens]
    p0 = [torch.randn(80, t, generator=gi).to(dev) for t in lens]

    def step(prec=a.precision, n=a.n_iters):
        return batching.attack_many("emb", [model_dev], vc, at, a.eps, n, ptb0s=p0, precision=prec, max_batch=B,
                                    ragged=not a.bucketed)
    # heartbeat on stderr: a per-length-bucket step (hundreds of single-utterance buckets) runs minutes
    # without output
    import threading
    hb_stop = threading.Event()

    def heartbeat():
        t_hb = time.perf_counter()
        while not hb_stop.wait(30.0):
            print(f"bench --lengths: running ({time.perf_counter() - t_hb:.0f} s)", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, None)
    hb_stop.set()
    assert all(torch.isfinite(o).all() for o in out)
    frames = sum(lens_all)
    roof = None
    if not a.no_roofline:
        ctx = avc_native.context_for(model_dev.speaker_encoder, dev)
        te = torch.cat([ctx.se_forward(x[None]) for x in at])
        order = sorted(range(len(lens)), key=lambda i: (-lens[i], i))   # attack_many's longest-first batch
        vo, po = [vc[i] for i in order], [p0[i] for i in order]
        ctx.ktime_start()
        ctx.emb_attack_ragged(vo, te[order], po, a.eps, KTIME_ITERS, precision=a.precision)
        kt = ctx.ktime_stop()
        ctx.set_profiling(True)
        ctx.emb_attack_ragged(vo, te[order], po, a.eps, PROF_ITERS, precision=a.precision)
        ms_iter, stats = ctx.profile()
        ctx.set_profiling(False)
        peak, unit = PEAK[a.precision]
        timed = {k: v for k, v in kt.items() if k in stats}
        base, (kn, kus) = max(timed.items(), key=lambda kv: kv[1][0] * kv[1][1])
        n, tot_ms, tot_fl = stats[base]
        achieved = (tot_fl / n) / (kus * 1e-6) / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4), "traffic": None, "kernel": base, "avg_launch_ms": round(kus * 1e-3, 5),
                "timing": f"in-graph device wall-clock stamps (avc_ktime), {kn} launches over {KTIME_ITERS} iterations",
                "flop_per_launch": tot_fl / n,
                "in_graph": {k: {"launches_per_iter": v[0] / KTIME_ITERS, "avg_ms": round(v[1] * 1e-3, 5)}
                             for k, v in kt.items()},
                "per_kernel": {k: {"launches_per_iter": v[0] / PROF_ITERS, "avg_ms": round(v[1] / v[0], 4)}
                               for k, v in stats.items()}}
        ppath = os.path.join(ROOT, "profiles", "pmc.json")
        if os.path.exists(ppath):
            rec = json.load(open(ppath)).get(f"emb_lengths_{lo}_{hi}", {}).get(base)
            if rec is not None:
                ver = avc_native.lib().avc_version().decode()
                roof.update(traffic=rec["traffic"], mfma_util=rec["mfma_util"], pmc_source=rec["source"],
                            pmc_src=rec.get("src"),
                            pmc_stale=rec.get("src") is None or ("src=" + rec["src"]) not in ver)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_lengths({k: v.detach().cpu() for k, v in model.state_dict().items()}, lens[:8],
                                   a.cpu_seconds, threads, frames / total)
    if rank == 0:
        value = total * a.steps / elapsed
        print(json.dumps({
            "metric": f"defended utts/sec @ n_iters={a.n_iters} eps={a.eps} emb-attack, utterance lengths uniform in "
                      f"[{lo}, {hi}] frames; 1/2/4/8 MI355X", "value": round(value, 3), "unit": "utts/s",
            "frames_per_s": round(frames * a.steps / elapsed, 1), "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.precision, "data": "synthetic",
            "config": {"workload": f"emb_attack of B={B}/GPU utterances, lengths uniform in [{lo}, {hi}] (seed 2; mean "
                                   f"{frames / total:.1f} frames), adv_tgt of their own lengths, n_iters={a.n_iters}, "
                                   f"eps={a.eps}; " + ("per-length buckets (batching.attack_many)" if a.bucketed else
                                                       "one ragged batch per GPU (batching.attack_many(ragged=True))"),
                       "batch_per_gpu": B, "lengths": [lo, hi], "mean_frames": round(frames / total, 2),
                       "n_iters": a.n_iters, "eps": a.eps,
                       "parallelism": f"dp{world} (independent utterance shards, no collective)"},
            "roofline": roof, "cpu_baseline": cpu, "libavc": avc_native.lib().avc_version().decode()}), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.cpu_worker > 0:
        return cpu_worker(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(a))
    if a.dry_run:
        return main_dry_run(a)
    if a.attack == "pm":
        return main_pm(a)
    if a.attack == "mel2wav":
        return main_mel2wav(a)
    if a.lengths:
        if a.attack != "emb":
            raise SystemExit("--lengths measures the emb attack")
        return main_lengths(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max only: no RCCL in the process

    import attack_utils
    import avc_native
    import models
    import shard

    torch.manual_seed(0)
    model = models.AdaInVC(FULL_CFG)           # random-init weights of the AdaIN-VC architecture
    model_dev = model.to(dev)
    B, T = a.batch, a.frames
    g = torch.Generator().manual_seed(1)
    total = B * world
    vc_all = torch.randn(total, 80, T, generator=g)
    at_all = torch.randn(total, 80, T, generator=g)
    p0_all = torch.randn(total, 80, T, generator=torch.Generator().manual_seed(123))
    sl = shard.shard_slice(total, rank, world)
    src_all = torch.randn(total, 80, T, generator=g)
    vc, at, p0, src = (t[sl].contiguous().to(dev) for t in (vc_all, at_all, p0_all, src_all))
    del vc_all, at_all, p0_all, src_all

    def step(prec=a.precision):
        if a.attack == "emb":
            return attack_utils.emb_attack(model_dev, vc, at, a.eps, a.n_iters, ptb0=p0, precision=prec)
        fn = attack_utils.e2e_attack if a.attack == "e2e" else attack_utils.fb_attack
        return fn(model_dev, src, vc, at, a.eps, a.n_iters, ptb0=p0, precision=prec)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, None)
    assert torch.isfinite(out).all()

    fp32_cmp = None
    if a.precision != "fp32" and not a.no_fp32_compare:
        # the exact-fp32 path on the same workload (one untimed warm-up, one timed step)
        step("fp32")
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        out32 = step("fp32")
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        e32 = shard.max_over_ranks(time.perf_counter() - t1, dist, None)
        fp32_cmp = {"value": round(total / e32, 3), "ms_per_step": round(e32 * 1e3, 3),
                    "max_abs_diff_vs_bf16": float((out32 - out).detach().abs().max())}

    roof = None
    flop_utt_iter = FLOP_PER_UTT_ITER[a.attack] * T / 128     # replaced by the library's count below
    if not a.no_roofline:
        if a.attack == "emb":
            ctx = avc_native.context_for(model_dev.speaker_encoder, dev)
        else:
            ctx = avc_native.vc_context_for(model_dev, dev)
        # the hot kernels' durations INSIDE the captured graph replay, no profiler attached: device
        # wall-clock stamps per workgroup (avc_ktime), over one more attack of the timed step's n_iters (the
        # persistent emb kernel's launch span depends on its length: clock ramp-up is amortised over it)
        # (right after the timed region: same workspace, same graphs)
        kti = a.n_iters
        ctx.ktime_start()
        if a.attack == "emb":
            ctx.emb_attack(vc, at, p0, a.eps, kti, precision=a.precision)
        else:
            ctx.vc_attack(a.attack, src, vc, at, p0, a.eps, kti, precision=a.precision)
        kt = ctx.ktime_stop()
        # per-launch FLOPs and the eager HIP kernel-timestamp durations (each kernel launched alone)
        ctx.set_profiling(True)
        if a.attack == "emb":
            ctx.emb_attack(vc, at, p0, a.eps, PROF_ITERS, precision=a.precision)
        else:
            ctx.vc_attack(a.attack, src, vc, at, p0, a.eps, PROF_ITERS, precision=a.precision)
        ms_iter, stats = ctx.profile()
        ctx.set_profiling(False)
        flop_utt_iter = ctx.prof_flop_per_iter / B
        eager = {k: (k, v) for k, v in stats.items()}
        timed = {k: v for k, v in kt.items() if k in eager}
        peak, unit = PEAK[a.precision]
        atk = "se_attack_fused<bf16>"
        per_iter = None
        if atk in kt:
            # the persistent emb attack: ONE launch ran all kti iterations.  Its unit of
            # work is one iteration -- the forward (+ fused head) and backward passes whose FLOPs the per-pass
            # profile below counts -- so achieved = FLOPs per iteration / launch span per iteration
            kn, kus = kt[atk]
            passes = [k for k in ("se_fwd_fused<bf16>", "se_bwd_fused<bf16>") if k in stats]
            fl_it = sum(stats[k][2] for k in passes) / PROF_ITERS
            per_iter = kti * kn
            name, n, tot_fl = atk, 1, fl_it
            tot_ms = sum(stats[k][1] for k in passes) / PROF_ITERS   # the per-pass launches' eager time per iteration
            avg_ms = kus * 1e-3 * kn / per_iter
            how = (f"in-graph device wall-clock stamps (avc_ktime): {kn} persistent launch(es) of {kti} "
                   f"iterations, per iteration")
        elif timed:   # dominant kernel by in-graph time per iteration
            base, (kn, kus) = max(timed.items(), key=lambda kv: kv[1][0] * kv[1][1])
            name, (n, tot_ms, tot_fl) = eager[base]
            avg_ms = kus * 1e-3
            how = f"in-graph device wall-clock stamps (avc_ktime), {kn} launches over {kti} iterations"
        else:       # no stamped kernel on this path: the eager per-launch HIP-event timing
            name, (n, tot_ms, tot_fl) = max(stats.items(), key=lambda kv: kv[1][1])
            avg_ms = tot_ms / n
            how = "eager per-launch HIP kernel-timestamp events"
        achieved = (tot_fl / n) / (avg_ms * 1e-3) / 1e12
        e_ms = tot_ms / n
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4), "traffic": None, "kernel": name,
                "avg_launch_ms": round(avg_ms, 5), "timing": how, "flop_per_launch": tot_fl / n,
                "avg_launch_ms_eager": round(e_ms, 5),
                "frac_eager": round((tot_fl / n) / (e_ms * 1e-3) / 1e12 / peak, 4),
                "iter_ms_profiled": round(ms_iter, 4),
                "in_graph": {k: {"launches_per_iter": v[0] / kti, "avg_ms": round(v[1] * 1e-3, 5),
                                 **({"tflops": round(eager[k][1][2] / eager[k][1][0] / (v[1] * 1e-6) / 1e12, 2)}
                                    if k in eager else {})} for k, v in kt.items()},
                "per_kernel": {k: {"launches_per_iter": v[0] / PROF_ITERS, "avg_ms": round(v[1] / v[0], 4),
                                   "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 2)} for k, v in stats.items()}}
        if per_iter:
            roof.update(per_iteration=True, avg_launch_ms=round(kus * 1e-3, 4), iters_per_launch=kti,
                        avg_iter_ms=round(avg_ms, 5), flop_per_iteration=tot_fl,
                        avg_launch_ms_eager=None, frac_eager=round(tot_fl / (tot_ms * 1e-3) / 1e12 / peak, 4),
                        iter_ms_eager_passes=round(tot_ms, 5))
            roof.pop("flop_per_launch", None)
        # HBM bytes and normalised MFMA utilisation of the same kernel from the committed
        # rocprofv3 PMC passes (scripts/pmc_fused.sh -> scripts/fz_summary.py -> profiles/pmc.json):
        # PMC counters cannot be read inside this process
        ppath = os.path.join(ROOT, "profiles", "pmc.json")
        key = a.attack + ("_fp32" if a.precision == "fp32" else "") + ("" if T == 128 else f"_T{T}")
        if os.path.exists(ppath):
            rec = json.load(open(ppath)).get(key, {}).get(name)
            if rec is not None:
                ipl = rec.get("iters_per_launch", 1) if per_iter else 1   # persistent kernel: per iteration
                roof["traffic"] = rec["traffic"] / ipl if rec["traffic"] is not None else None
                roof["mfma_util"] = rec["mfma_util"]
                roof["pmc_source"] = rec["source"]
                roof["pmc_median_us"] = rec["median_us"]
                if per_iter:
                    roof["pmc_iters_per_launch"] = ipl
                    roof["pmc_median_us_per_iter"] = round(rec["median_us"] / ipl, 2)
                # counters of another build than the one measured here are flagged, not passed off
                ver = avc_native.lib().avc_version().decode()
                roof["pmc_src"] = rec.get("src")
                roof["pmc_stale"] = rec.get("src") is None or ("src=" + rec["src"]) not in ver

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(model, a.cpu_seconds, a.attack, a.cpu_procs)

    if rank == 0:
        ms = elapsed / a.steps * 1e3
        value = total * a.steps / elapsed
        base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
        metric = base["metric"] if a.attack == "emb" else \
            f"defended utts/sec @ n_iters={a.n_iters} eps={a.eps} {a.attack}-attack; 1/2/4/8 MI355X"
        cfg_no = {"emb": 1, "e2e": 2, "fb": 3}[a.attack]
        fl = flop_utt_iter
        line = {
            "metric": metric, "value": round(value, 3), "unit": "utts/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.precision, "data": "synthetic",
            "config": {"workload": f"{a.attack}_attack B={B}/GPU T={T} n_iters={a.n_iters} eps={a.eps} "
                                   f"(BASELINE configs[{cfg_no}]; AdaIN-VC, random init seed 0)",
                       "batch_per_gpu": B, "frames": T, "n_iters": a.n_iters, "eps": a.eps,
                       "parallelism": f"dp{world} (independent utterance shards, no collective)"},
            "roofline": roof, "cpu_baseline": cpu, "fp32": fp32_cmp,
            "libavc": avc_native.lib().avc_version().decode(),
            "flop_per_utt_iter": fl,
            "tflops_whole_step": round(fl * a.n_iters * total * a.steps / elapsed / 1e12, 2),
        }
        if roof is not None:
            # the unprofiled graph-replayed loop's algorithmic rate over the peak, next to the
            # per-kernel (HIP-event, instrumented) frac above: the in-loop figure has no profiler
            # stretch, and the per-kernel times summed exceed ms_per_step / n_iters by that stretch
            pk = PEAK[a.precision][0]
            roof["frac_in_loop_whole_step"] = round(line["tflops_whole_step"] / world / pk, 4)
            roof["iter_ms_in_loop"] = round(ms / a.n_iters, 5)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
