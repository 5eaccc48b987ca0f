"""bench.py honours --gpus: a world size that disagrees with --gpus is an error, not a silent
1-GPU run (checked before anything touches a GPU, so it runs here)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 1 but WORLD_SIZE=2" in (r.stderr + r.stdout)
