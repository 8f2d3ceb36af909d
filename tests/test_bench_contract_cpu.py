"""bench.py's launch contract, checked without a GPU: `--gpus N` with fewer visible GPUs fails
loudly (never times fewer GPUs than requested), a torchrun WORLD_SIZE that disagrees with
--gpus is refused, and with no GPU at all the single-GPU run exits with a clear message instead
of timing a CPU fallback."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_more_gpus_than_visible():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "refusing to time fewer GPUs" in (r.stdout + r.stderr)


def test_bench_refuses_world_size_mismatch():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=4" in (r.stdout + r.stderr)


def test_bench_needs_a_gpu():
    r = _run(["--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "needs a GPU" in (r.stdout + r.stderr)
