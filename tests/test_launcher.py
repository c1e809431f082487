"""`bench.py --gpus N` without a torch.distributed launcher starts N rank processes itself
(wab_gym_amd.shard.launch_ranks).  CPU tests: every child gets a distinct RANK / LOCAL_RANK,
the rendezvous variables torch.distributed.run would set, rank 0's stdout comes back, and a
failing child's exit code is propagated (and does not leave the others hanging)."""
import json
import os
import subprocess
import sys
import time

from wab_gym_amd.shard import launch_ranks

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
d = {k: os.environ.get(k) for k in keys}
open(os.path.join(sys.argv[1], "rank%s.json" % d["RANK"]), "w").write(json.dumps(d))
if d["RANK"] == "0":
    print("not json")
    print(json.dumps({"rank0": True}))
"""


def test_launch_distinct_ranks(tmp_path):
    rc, out, codes = launch_ranks([sys.executable, "-c", CHILD, str(tmp_path)], 4)
    assert rc == 0 and codes == [0, 0, 0, 0]
    seen = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(4)]
    assert [int(d["RANK"]) for d in seen] == [0, 1, 2, 3]
    assert [int(d["LOCAL_RANK"]) for d in seen] == [0, 1, 2, 3]
    assert {d["WORLD_SIZE"] for d in seen} == {"4"} and {d["LOCAL_WORLD_SIZE"] for d in seen} == {"4"}
    assert {d["MASTER_ADDR"] for d in seen} == {"127.0.0.1"}
    assert len({d["MASTER_PORT"] for d in seen}) == 1
    assert out.splitlines()[-1] == '{"rank0": true}'


def test_launch_propagates_child_failure():
    # rank 1 fails at once; rank 0 would wait forever (a rank stuck at a barrier): the launch
    # must return rank 1's code and kill rank 0
    child = ("import os, sys, time\n"
             "r = int(os.environ['RANK'])\n"
             "if r == 1: sys.exit(7)\n"
             "time.sleep(600)\n")
    t0 = time.monotonic()
    rc, _, codes = launch_ranks([sys.executable, "-c", child], 2)
    assert rc == 7 and codes[1] == 7 and codes[0] != 0
    assert time.monotonic() - t0 < 60


def test_launch_timeout_kills_all():
    rc, _, codes = launch_ranks([sys.executable, "-c", "import time; time.sleep(600)"], 2, timeout=2)
    assert rc != 0 and all(c != 0 for c in codes)


def test_bench_refuses_more_ranks_than_gpus():
    # no GPU here: --gpus 2 must refuse (without --share-gpu) instead of silently timing one GPU
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu"],
                       capture_output=True, text=True, timeout=600,
                       env={k: v for k, v in os.environ.items()
                            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode != 0
    assert "--share-gpu" in r.stderr
    assert not r.stdout.strip()


def test_ranks_bind_distinct_devices():
    """One process per GPU: on an 8-GPU node ranks 0..7 bind devices 0..7, each its own; with
    fewer GPUs than ranks a rank without a GPU is refused unless the run shares them."""
    import pytest

    from wab_gym_amd.shard import device_for_rank

    assert [device_for_rank(r, 8) for r in range(8)] == list(range(8))
    assert [device_for_rank(r, 4) for r in range(4)] == [0, 1, 2, 3]
    assert [device_for_rank(r, 1, share_gpu=True) for r in range(2)] == [0, 0]
    with pytest.raises(SystemExit):
        device_for_rank(1, 1)
    with pytest.raises(SystemExit):
        device_for_rank(0, 0)
