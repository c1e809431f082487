"""One rank of tests/test_gpu_multiprocess.py (started by wab_gym_amd.shard.launch_ranks, the
launcher `bench.py --gpus N` uses): its shard of env ids [r*B, (r+1)*B) on the GPU, 36 env.step
calls then one 64-step env.rollout, every step's obs (planes bit-packed), scalars, reward and
done saved for the parent to compare with one oracle batch of N*B envs.  A gloo group carries
the barrier and an all-gather of the shard bases (the bench's collectives; no RCCL)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main(out_dir, B, T_step, T_roll):
    import numpy as np
    import torch
    import torch.distributed as dist

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.shard import all_gather_objects, env_id_base, rank_info

    rank, world, local = rank_info()
    torch.cuda.set_device(local % torch.cuda.device_count())
    dist.init_process_group("gloo")
    env = BatchedWolvesAndBushesEnv(None, num_envs=B, seed=0x5EED, device="cuda", validate_actions=False,
                                    env_id_base=env_id_base(rank, B))
    bases = all_gather_objects(env.env_id_base)
    assert bases == [r * B for r in range(world)], bases
    env.reset()
    acts = np.random.RandomState(7).randint(5, size=(T_step + T_roll, world * B)).astype(np.int8)
    acts = acts[:, rank * B:(rank + 1) * B]
    bits, scal, rew, done = [], [], [], []
    for t in range(T_step):
        obs, r, d, _ = env.step(torch.as_tensor(acts[t], device=env.device))
        bits.append(np.packbits(env._obs["planes"].cpu().numpy().reshape(B, -1), axis=1))
        scal.append(env._obs["scalars"].cpu().numpy())
        rew.append(r.cpu().numpy())
        done.append(d.cpu().numpy().astype(np.uint8))
    planes, sc, r, d = env.rollout(torch.as_tensor(acts[T_step:], device=env.device))
    bits.extend(np.packbits(planes.cpu().numpy().reshape(T_roll, B, -1), axis=2))
    scal.extend(sc.cpu().numpy())
    rew.extend(r.cpu().numpy())
    done.extend(d.cpu().numpy())
    c = env.counters()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), bits=np.stack(bits), scalars=np.stack(scal),
             reward=np.stack(rew), done=np.stack(done), steps=c["steps"], overflow=c["wolf_overflow"],
             device=str(torch.cuda.current_device()))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
