"""One process per GPU, launched by the bench scripts themselves.

    rc = launch.relaunch(n, script, argv)   # parent: before ANY GPU call
    ctx = launch.init_ranks(n, backend)      # in every rank

`relaunch` starts `python -m torch.distributed.run --nproc-per-node n
--master-addr 127.0.0.1 ...` as a CHILD process (never exec: the parent must
not have touched the GPU, and it only waits for the children and returns
their exit code).  When the script already runs under torchrun (WORLD_SIZE is
set, e.g. the driver's own launch) nothing is relaunched.

`init_ranks` binds local rank r to device r, joins the process group (RCCL
over xGMI for "nccl", gloo for CPU-only runs) and checks that the world size
is the one asked for, so `--gpus 8` can never silently measure one rank.
There is no data-path collective: the shards are disjoint; the group carries
only the harness barrier and the per-rank timings.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def under_launcher():
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def relaunch(n, script, argv, extra_env=None):
    """Run `script argv` as n ranks under torch.distributed.run; returns the
    exit code, or None when no relaunch is needed (n == 1 or already a rank)."""
    if n <= 1 or under_launcher():
        return None
    env = os.environ.copy()
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    if extra_env:
        env.update(extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", script] + list(argv)
    return subprocess.run(cmd, env=env).returncode


class Ranks:
    def __init__(self, world, rank, local, device, backend, pg=None):
        self.world, self.rank, self.local, self.device, self.backend = world, rank, local, device, backend
        # a process group exists: world > 1, or SSTC_PG_SINGLE at world 1
        self.pg = world > 1 if pg is None else pg

    @property
    def on(self):
        return self.pg

    def barrier(self):
        if self.on:
            dist.barrier()

    def _t(self, v):
        dev = self.device if self.backend == "nccl" else None
        return torch.tensor([float(x) for x in v], dtype=torch.float64, device=dev)

    def max(self, value):
        if not self.on:
            return float(value)
        t = self._t([value])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, value):
        if not self.on:
            return float(value)
        t = self._t([value])
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def gather(self, values):
        """Every rank's list of floats (same length on all ranks), rank order."""
        if not self.on:
            return [list(map(float, values))]
        t = self._t(values)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def close(self):
        if self.on:
            dist.barrier()
            dist.destroy_process_group()


def init_ranks(n_expected, backend="nccl"):
    """Join the job as one rank.  backend "nccl" (RCCL): bind LOCAL_RANK to its
    GPU; "gloo": CPU only (plumbing tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_expected:
        raise SystemExit(f"asked for {n_expected} ranks but WORLD_SIZE={world}")
    device = None
    if backend == "nccl":
        if torch.cuda.device_count() < world:
            raise SystemExit(f"{world} ranks need {world} GPUs, {torch.cuda.device_count()} visible")
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    # SSTC_PG_SINGLE=1 under a launcher: a one-rank process group as well, so
    # the collective path (RCCL init with device_id, barrier, max / sum /
    # gather) runs on a one-GPU box (tests/test_gpu_bench_rank.py)
    pg = world > 1 or (under_launcher() and os.environ.get("SSTC_PG_SINGLE") == "1")
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == n_expected
        print(f"[sstc] process group: {dist.get_backend()}, world {dist.get_world_size()}", file=sys.stderr,
              flush=True)
    return Ranks(world, rank, local, device, backend, pg)
