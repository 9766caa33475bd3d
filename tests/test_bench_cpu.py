"""bench.py launcher contract on the CPU: an external launcher's WORLD_SIZE must equal --gpus
(checked before anything imports torch or touches a GPU)."""
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in p.stderr
