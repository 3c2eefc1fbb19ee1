"""CPU (gloo, world_size 2): the multi-process sharding path of bench.py --
contiguous utterance shards, max-over-ranks timing, host-side gather -- with the
CPU oracle standing in for the per-rank compute (no GPU here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def test_shard_slice_covers_exactly():
    for total in (0, 1, 7, 256, 2048, 2049):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                sl = shard_slice_list(total, r, world)
                got.extend(sl)
            assert got == list(range(total)), (total, world)
            sizes = [len(shard_slice_list(total, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def shard_slice_list(total, r, world):
    sl = shard.shard_slice(total, r, world)
    return list(range(sl.start, sl.stop))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import json
    from conftest import GOLDEN
    from oracle import adain_vc as oracle
    z = np.load(os.path.join(GOLDEN, "small_T32.npz"))
    cfg = json.loads(str(z["config"]))
    w = oracle.Weights({k[2:]: z[k] for k in z.files if k.startswith("w/")})
    g = torch.Generator().manual_seed(3)
    x = torch.randn(total, 80, 32, generator=g).numpy()
    sl = shard.shard_slice(total, rank, world)
    emb = np.concatenate([oracle.se_forward(w, cfg["SpeakerEncoder"], x[b:b + 1])[0]
                          for b in range(sl.start, sl.stop)]) if sl.stop > sl.start else np.zeros((0, 32), np.float32)
    full = shard.gather_shards(torch.from_numpy(emb), total, dist)
    t = shard.max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        q.put((full.numpy(), t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [5, 6])
def test_gloo_two_ranks_gather_and_max(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: the same per-utterance oracle in one process
    import json
    from conftest import GOLDEN
    from oracle import adain_vc as oracle
    z = np.load(os.path.join(GOLDEN, "small_T32.npz"))
    cfg = json.loads(str(z["config"]))
    w = oracle.Weights({k[2:]: z[k] for k in z.files if k.startswith("w/")})
    x = torch.randn(total, 80, 32, generator=torch.Generator().manual_seed(3)).numpy()
    ref = np.concatenate([oracle.se_forward(w, cfg["SpeakerEncoder"], x[b:b + 1])[0] for b in range(total)])
    assert np.array_equal(full, ref)
    assert t == 2.0


def _bench(*args, timeout=240):
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), capture_output=True,
                          text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("world,batch", [(2, 8), (3, 5)])
def test_bench_launcher_dry_run(world, batch):
    """`python bench.py --gpus N` without torchrun starts the N rank processes itself (gloo
    here: --dry-run computes no attack); rank 0 prints one JSON line whose shards cover the
    global batch exactly."""
    import json
    r = _bench("--gpus", str(world), "--dry-run", "--batch", str(batch), "--frames", "16", "--steps", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["global_batch"] == batch * world
    assert out["shard_sizes"] == [batch] * world


def test_bench_refuses_missing_gpus():
    """No silent single-GPU number: --gpus 2 with fewer visible GPUs (none here) fails loudly."""
    r = _bench("--gpus", "2", "--steps", "1", timeout=120)
    assert r.returncode != 0
    assert "GPU(s) are visible" in (r.stderr + r.stdout)


def test_launcher_gpu_count_never_initialises_hip(tmp_path, monkeypatch):
    """bench.py's launcher counts GPUs from sysfs (KFD topology + accessible render nodes, narrowed by the
    *_VISIBLE_DEVICES variables) and never calls into torch.cuda: a process that has initialised HIP must
    not fork the rank processes."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    def boom(*a, **k):
        raise AssertionError("the launcher's GPU count reached torch.cuda / HIP")
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    nodes.mkdir()
    dri.mkdir()
    # node 0: a CPU; nodes 1-3: GPUs with render minors 128-130, of which 130 is not in this "container"
    for i, (gid, minor) in enumerate([(0, None), (1111, 128), (2222, 129), (3333, 130)]):
        (nodes / str(i)).mkdir()
        txt = f"cpu_cores_count 8\ngpu_id {gid}\n" + (f"drm_render_minor {minor}\n" if minor else "")
        (nodes / str(i) / "properties").write_text(txt)
    for minor in (128, 129):
        (dri / f"renderD{minor}").write_text("")
    assert bench.visible_gpu_count(str(nodes), str(dri)) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_gpu_count(str(nodes), str(dri)) == 1
    assert bench.visible_gpu_count(str(tmp_path / "absent"), str(dri)) == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    # the launcher refuses more ranks than visible GPUs, through the same count
    monkeypatch.setattr(bench, "KFD_NODES", str(tmp_path / "absent"))
    monkeypatch.setattr(bench, "visible_gpu_count", lambda nodes=None, dev_dir=None: 0)

    class A:
        dry_run, gpus = False, 2
    with pytest.raises(SystemExit, match="only 0 GPU"):
        bench.launch_ranks(A())
