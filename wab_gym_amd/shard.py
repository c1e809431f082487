"""Multi-GPU sharding of the env batch: independent shards, no collective.

Rank r of N owns global env ids [r*B, (r+1)*B).  Every random draw is keyed by the global
id, so the union of the shards reproduces one batch of N*B envs exactly (tested).  The
only collectives are out of the data path and run over a CPU (gloo) process group: a
barrier around the timed region, a MAX reduction of the elapsed time and a gather of the
per-rank figures (bench.py).  RCCL is never initialised.
"""
from __future__ import annotations

import os
import socket
import subprocess
import threading
import time


def free_port(host="127.0.0.1") -> int:
    """An unused TCP port on `host` for the rendezvous."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def launch_ranks(cmd, n, env=None, master_port=None, timeout=None):
    """Run `cmd` (an argv list) as `n` fresh rank processes, one per GPU, the way
    `torch.distributed.run --nproc-per-node n --master-addr 127.0.0.1` would: child r gets
    RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n and MASTER_ADDR/PORT.  The caller
    must not have touched the GPU (the children are started, not exec'd).  Returns
    (exit code, rank 0's stdout, every rank's exit code): the exit code is that of the first
    child to fail on its own (lowest rank among simultaneous failures; 0 when all succeed).
    If one child fails the rest are killed, so a rank stuck at a barrier cannot hang the
    launch; on `timeout` (seconds) every child still running is killed and the code is -9."""
    base = dict(os.environ if env is None else env)
    port = master_port or free_port()
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout is captured (it carries the JSON line); the others inherit ours
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else None))
    out0 = []

    def pump():
        for line in procs[0].stdout:
            out0.append(line.decode(errors="replace"))
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    codes = [None] * n
    t_end = None if timeout is None else time.monotonic() + timeout
    first_failure = 0
    try:
        while any(c is None for c in codes):
            for r, p in enumerate(procs):
                if codes[r] is None:
                    codes[r] = p.poll()
            failed = [c for c in codes if c not in (None, 0)]
            late = t_end is not None and time.monotonic() > t_end
            if failed or late:
                first_failure = failed[0] if failed else -9
                break
            time.sleep(0.05)
    finally:
        # whatever ends the wait (a failure, the timeout, an exception or KeyboardInterrupt in
        # this process), no child that may hold the GPU is left running
        for r, p in enumerate(procs):
            if codes[r] is None:
                if p.poll() is None:
                    p.kill()
                codes[r] = p.wait()
    th.join(timeout=10)
    return first_failure, "".join(out0), codes


def rank_info():
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def env_id_base(rank: int, batch_per_rank: int) -> int:
    return rank * batch_per_rank


def _initialised():
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def max_over_ranks(value: float) -> float:
    """MAX of a per-rank float over the default (CPU, gloo) process group; identity when not
    initialised."""
    import torch
    import torch.distributed as dist

    if not _initialised():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_objects(obj):
    """Every rank's `obj`, in rank order (a one-element list when not initialised)."""
    import torch.distributed as dist

    if not _initialised():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def device_for_rank(local_rank, n_devices, share_gpu=False):
    """The GPU index rank `local_rank` binds (one process per GPU: LOCAL_RANK r -> device r).  With
    fewer visible GPUs than ranks it raises unless share_gpu (the 1-GPU rehearsal of N > 1, ranks
    then share device local_rank % n_devices)."""
    if n_devices < 1:
        raise SystemExit("no GPU visible")
    if local_rank >= n_devices and not share_gpu:
        raise SystemExit("rank %d has no GPU of its own (%d visible); pass --share-gpu" % (local_rank, n_devices))
    return local_rank % n_devices
