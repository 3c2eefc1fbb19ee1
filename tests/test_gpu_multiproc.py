"""libavc in more than one process: two rank processes (gloo, both on the box's one GPU) each
attack their contiguous shard through the HIP path and gather on the host -- bench.py's
multi-GPU data path with real kernels instead of the CPU stand-in of test_distributed.py.
The gathered result must equal one process attacking the whole batch bitwise (per-utterance
arithmetic never depends on the batch: DESIGN.md 5)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gpu_mp_worker as W  # noqa: E402

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind,total", [("emb", 5), ("fb", 3)])
def test_two_rank_processes_match_single(tmp_path, kind, total):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    T, n, prec = 128, 6, "bf16"
    out = str(tmp_path / "full.npy")
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_mp_worker.py"), kind, str(total),
                                       str(T), str(n), prec, out], env=env))
    codes = [p.wait(timeout=300) for p in procs]
    assert codes == [0, 0], codes
    got = np.load(out)
    vc, at, src, p0 = W.inputs(total, T)
    ref = W.run(kind, vc, at, src, p0, torch.device("cuda", 0), n, prec).detach().cpu().numpy()
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
