"""bench.py --gpus N without a launcher spawns its N rank processes itself
(the driver's scaling run may call `python3 bench.py --gpus 8` directly).

On this CPU container every rank gets as far as the rank setup (gloo process
group, RCCL unique id) and fails only where it opens its HIP device; the
parent must report every child, stop, and exit non-zero.  A --gpus that
disagrees with a launcher's WORLD_SIZE is refused before anything runs."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks_which_reach_device_open():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--shard-cells", "60", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=600,
                       env=_env(HIP_VISIBLE_DEVICES=""))
    err = r.stderr
    spawned = re.findall(r"\[bench\] spawned rank (\d)/2 pid (\d+)", err)
    assert sorted(int(s[0]) for s in spawned) == [0, 1], err[-3000:]
    up = re.findall(r"\[bench\] rank (\d)/2 pid (\d+) up", err)
    assert sorted(int(s[0]) for s in up) == [0, 1], err[-3000:]
    # the children are the spawned PIDs, not the parent
    assert {p for _, p in up} == {p for _, p in spawned}
    # no GPU here: the ranks fail at the device, after the rank setup
    assert r.returncode != 0
    assert "hipSetDevice" in err or "ROCm-capable device" in err or "xfk error" in err, err[-3000:]
    exited = re.findall(r"\[bench\] rank (\d) exited with (-?\d+)", err)
    assert sorted(int(e[0]) for e in exited) == [0, 1], err[-3000:]
    assert r.stdout.strip() == ""      # no JSON line from a failed run


def test_gpus_mismatching_world_size_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--steps", "1"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "does not match" in r.stderr
    assert "spawned" not in r.stderr
