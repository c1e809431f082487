"""The multi-process GPU path: rank processes started by the launcher
`bench.py --gpus N` uses (wab_gym_amd.shard.launch_ranks), each stepping its own shard of
global env ids on the GPU (here both share the box's one GPU), and the concatenated shards
compared with one oracle batch of all env ids, bit for bit, every step (obs planes, scalars,
reward, done) through both env.step and env.rollout."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_rank_processes_match_one_oracle_batch(tmp_path):
    from oracle.oracle import OracleBatch
    from wab_gym_amd.shard import launch_ranks

    world, B, T_step, T_roll = 2, 4096, 36, 64
    rc, out, codes = launch_ranks([sys.executable, os.path.join(HERE, "mp", "rank_child.py"), str(tmp_path),
                                   str(B), str(T_step), str(T_roll)], world, timeout=240)
    assert rc == 0, (rc, codes)
    shards = [np.load(tmp_path / ("rank%d.npz" % r)) for r in range(world)]
    for z in shards:
        assert int(z["steps"]) == B * (T_step + T_roll) and int(z["overflow"]) == 0
    orc = OracleBatch(None, world * B, 0x5EED, 0)
    orc.reset()
    acts = np.random.RandomState(7).randint(5, size=(T_step + T_roll, world * B)).astype(np.int8)
    for t in range(T_step + T_roll):
        op, of, orl, ost, orew, odone = orc.step(acts[t], nthreads=16)
        want_bits = np.packbits(op.reshape(world * B, -1), axis=1)
        got = lambda k: np.concatenate([z[k][t] for z in shards], axis=-1 if k == "scalars" else 0)  # noqa: E731
        assert np.array_equal(got("bits"), want_bits), t
        assert np.array_equal(got("scalars"), np.stack([of, orl, ost])), t
        assert np.array_equal(got("reward"), orew), t
        assert np.array_equal(got("done"), odone), t
