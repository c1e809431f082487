"""N>1 path on CPU (gloo, world_size 2): shards keyed by global env id reproduce one batch,
and the timing reduction is a MAX over ranks.  The GPU bench uses the same helpers over the
same CPU (gloo) process group: RCCL is never initialised."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

B, T = 96, 60


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    from oracle.oracle import OracleBatch
    from wab_gym_amd.shard import all_gather_objects, env_id_base, max_over_ranks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = OracleBatch(None, B, 0x5EED, env_id_base(rank, B))
    orc.reset()
    acts = np.random.RandomState(11).randint(5, size=(T, world * B))
    planes, rewards = [], []
    for t in range(T):
        p, _, _, _, r, _ = orc.step(acts[t, rank * B:(rank + 1) * B])
        planes.append(p.copy())
        rewards.append(r.copy())
    mine = torch.as_tensor(np.stack(planes))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    rg = [torch.zeros(T, B) for _ in range(world)]
    dist.all_gather(rg, torch.as_tensor(np.stack(rewards)))
    tmax = max_over_ranks(1.0 + rank)
    per_rank = all_gather_objects({"rank": rank, "base": env_id_base(rank, B)})
    assert per_rank == [{"rank": r, "base": r * B} for r in range(world)]
    if rank == 0:
        np.save(os.path.join(out_dir, "planes.npy"), torch.cat(gathered, dim=1).numpy())
        np.save(os.path.join(out_dir, "reward.npy"), torch.cat(rg, dim=1).numpy())
        np.save(os.path.join(out_dir, "tmax.npy"), np.array([tmax]))
    dist.destroy_process_group()


def test_two_rank_shards_equal_one_batch(tmp_path):
    from oracle.oracle import OracleBatch

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    planes = np.load(tmp_path / "planes.npy")
    reward = np.load(tmp_path / "reward.npy")
    assert float(np.load(tmp_path / "tmax.npy")[0]) == 2.0
    one = OracleBatch(None, world * B, 0x5EED, 0)
    one.reset()
    acts = np.random.RandomState(11).randint(5, size=(T, world * B))
    for t in range(T):
        p, _, _, _, r, _ = one.step(acts[t])
        assert np.array_equal(planes[t], p), t
        assert np.array_equal(reward[t], r), t
