"""Multi-process GPU checks (2 ranks sharing the test GPU): the one-shot IPC all-reduce kernel
(eager and inside a replayed hipGraph) and tensor-parallel Llama (column/row-parallel kernels +
one-shot all-reduce + vocab-parallel LM head) against TP=1.  Each runs under torchrun in a child
process with its own timeout."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(script, extra_env=None, timeout=240, nproc=2):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(_port()), os.path.join(ROOT, "tools", script)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def test_oneshot_allreduce_two_ranks():
    rc, out = _torchrun("ar_check.py")
    assert rc == 0 and "AR_CHECK PASS" in out, out[-3000:]


def test_tensor_parallel_llama_two_ranks():
    rc, out = _torchrun("tp_check.py", {"VWA_DIST_BACKEND": "gloo"})
    assert rc == 0 and "TP_CHECK PASS" in out, out[-3000:]


def test_tp_brain_continuous_batching_two_ranks():
    """brain/tp_engine.py on the GPU kernels: 4 concurrent requests on a TP=2 group decode together
    in lockstep (chained layers with in-launch all-reduce rounds, vocab-parallel sampling)."""
    rc, out = _torchrun("tp_brain_check.py", {"VWA_DIST_BACKEND": "gloo"}, timeout=280)
    assert rc == 0 and "TP_BRAIN_CHECK PASS" in out, out[-3000:]


def test_rccl_backend_collectives():
    """RCCL itself (backend "nccl" = RCCL on ROCm) -- round 5 never initialised it: all-reduce of
    decode- and prefill-sized bf16 messages, broadcast and a metrics all-gather on the GPU.  One
    rank: RCCL refuses two ranks on one device, and 8-GPU runs are the driver's."""
    rc, out = _torchrun("rccl_check.py", nproc=1, timeout=200)
    assert rc == 0 and "RCCL_CHECK PASS" in out, out[-3000:]


def test_tp_preflight_on_shared_device():
    """parallel/custom_ar.py preflight at group start (peer-access report by PCI id, one all-reduce
    self-test with a deadline) runs inside every 2-rank check above; this one asserts its report:
    two ranks on ONE device need no P2P mapping."""
    rc, out = _torchrun("ar_check.py", {"VWA_AR_CHECK_REPORT": "1"})
    assert rc == 0 and "AR_CHECK PASS" in out and "PREFLIGHT {'pci':" in out, out[-3000:]
