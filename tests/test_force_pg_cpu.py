"""``init_distributed(force_pg=True)`` on CPU: a one-rank gloo group with every collective forced on
must give bitwise the no-collective result (tests/_rccl_check.py, the GPU test's script, on gloo)."""
import os
import subprocess
import sys

from ._mp import child_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_force_pg_one_rank_gloo_cpu():
    env = child_env(OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="")
    env.pop("MASTER_ADDR", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "_rccl_check.py"), "gloo"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "RCCL_CHECK_PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
