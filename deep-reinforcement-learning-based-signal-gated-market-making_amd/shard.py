"""Population shards over ranks and the one exchange per generation.

The reference evaluates the whole population in one process
(Env/drl_engine.py:104-115, Pool.starmap).  Here rank r of a world of W owns
the contiguous shard [r*n, min(P, (r+1)*n)) with n = ceil(P / W), regenerates
its own genomes from the replicated master (counter-based, no genome traffic),
rolls them out, and writes its results into a fixed-size per-rank record:

    f64 fitness[2n]   train results at [0, n), validation results at [n, 2n)
    i32 trades[2n]    same order
    -> 24 n bytes

One all-gather of the records (RCCL over xGMI; staged through host memory on
the gloo backend) gives every rank the same [W, 24n]-byte array, which
sgmm_ga_step reads in place: individual i's value is at byte offset
(i // n) * 24n + field offset + (i % n) * element size.  Every rank then runs
the identical step (argmax, master regeneration, sigma decay), so masters stay
identical without a broadcast.
"""
from __future__ import annotations

import numpy as np
import torch


def shard_capacity(P: int, world: int) -> int:
    return -(-int(P) // int(world)) if P > 0 else 0


def shard_bounds(P: int, rank: int, world: int):
    """Contiguous population shard of a rank: [i0, i1) (may be empty)."""
    n = shard_capacity(P, world)
    i0 = min(P, rank * n)
    return i0, min(P, i0 + n)


# field byte offsets within a record of capacity n: (offset, element size)
def field_layout(n: int):
    return {"train_f": (0, 8), "val_f": (8 * n, 8), "train_t": (16 * n, 4), "val_t": (20 * n, 4)}


def record_bytes(n: int) -> int:
    return 24 * n


def element_offset(i: int, n: int, field: str) -> int:
    """Byte offset of individual i's `field` in the gathered records (the
    addressing sgmm_ga_step implements with shard_n = n, shard_stride = 24n)."""
    off, size = field_layout(n)[field]
    return (i // n) * record_bytes(n) + off + (i % n) * size


class FitnessRecords:
    """The rank's record and the gathered records of all ranks.

    With K populations (n_pop) the record holds every population's shard:
    f64 fitness[K][2n] then i32 trades[K][2n] (24 K n bytes); population k's
    fields sit at k * 16n (fitness) and 16Kn + k * 8n (trades) -- K = 1 is the
    single-population layout above.

    with_val=False (validation of the best only, after the tell): training
    results alone, f64 fitness[K][n] then i32 trades[K][n] (12 K n bytes)."""

    def __init__(self, P: int, world: int, device, n_pop: int = 1, gather: bool | None = None,
                 with_val: bool = True, group_active: bool = True):
        # gather: keep a gathered buffer and exchange even at world 1 (the
        # sharded path rehearsed on one process); default: world > 1.
        # group_active: the session runs over a process group (DRLEngine(dist=False)
        # is one process even when a default group exists: the gather is then a copy)
        self.P, self.world, self.K = int(P), int(world), int(n_pop)
        self.sharded = bool(world > 1 if gather is None else gather)
        self.group_active = bool(group_active)
        if self.world > 1 and not self.group_active:
            raise ValueError("a world of several ranks needs a process group")
        self.with_val = bool(with_val)
        n = self.n = shard_capacity(P, world)
        K = self.K
        self.device = torch.device(device)
        per = 2 if self.with_val else 1  # results per individual slot
        self.rbytes = 12 * per * n  # one population's record
        self.rec = torch.zeros(K * self.rbytes, dtype=torch.uint8, device=self.device)
        f = self.rec[:8 * per * K * n].view(torch.float64)
        t = self.rec[8 * per * K * n:].view(torch.int32)
        self.f, self.t = f, t
        self.train = (f[:n], t[:n])
        self.val = (f[n:2 * n], t[n:2 * n]) if self.with_val else None
        self.both = (f, t)  # per population train then validation, for one fused launch
        self.gathered = torch.zeros(world * K * self.rbytes, dtype=torch.uint8, device=self.device) \
            if self.sharded else None
        self._host = None

    def all_gather(self, group=None):
        """The generation's one collective.  RCCL gathers device buffers
        directly; gloo (CPU tests, one-GPU rehearsals) goes through host memory."""
        import torch.distributed as dist
        if not self.sharded:
            return
        if not (self.group_active and dist.is_available() and dist.is_initialized()):
            # one process (no group, or the session opted out of it): the gather is a copy
            self.gathered.copy_(self.rec)
            return
        if self.device.type == "cuda" and dist.get_backend(group) == "gloo":
            if self._host is None:
                self._host = (torch.empty_like(self.rec, device="cpu"),
                              torch.empty_like(self.gathered, device="cpu"))
            src, dst = self._host
            src.copy_(self.rec)
            dist.all_gather_into_tensor(dst, src, group=group)
            self.gathered.copy_(dst)
        else:
            dist.all_gather_into_tensor(self.gathered, self.rec, group=group)

    def step_args(self):
        """(fit, trades, val_fit, val_trades, P, shard_n, shard_stride): the
        population arguments of sgmm_ga_step -- pointers into the gathered
        records, or the local record read contiguously when world == 1."""
        import ctypes
        n = self.n
        lay = field_layout(n)
        base = (self.gathered if self.sharded else self.rec).data_ptr()
        ptrs = tuple(ctypes.c_void_p(base + lay[k][0]) for k in ("train_f", "train_t", "val_f", "val_t"))
        shard = (n, record_bytes(n)) if self.sharded else (0, 0)
        return ptrs + (self.P,) + shard

    def multi_step_args(self):
        """(fit, trades, val_fit, val_trades, fit_pop_stride, trades_pop_stride,
        shard_n, shard_stride): the arguments of sgmm_ga_step_multi --
        population 0's field pointers into the gathered records (or the local
        record when world == 1) and the per-population byte strides."""
        import ctypes
        n, K = self.n, self.K
        base = (self.gathered if self.sharded else self.rec).data_ptr()
        offs = (0, 16 * K * n, 8 * n, 16 * K * n + 4 * n)  # train_f, train_t, val_f, val_t
        ptrs = tuple(ctypes.c_void_p(base + o) for o in offs)
        shard = (n, K * record_bytes(n)) if self.sharded else (0, 0)
        return ptrs + (16 * n, 8 * n) + shard

    def tell_args(self):
        """(fit, trades, fit_pop_stride, trades_pop_stride, shard_n, shard_stride):
        the arguments of sgmm_ga_tell_multi over the training results (either
        layout), gathered or local."""
        import ctypes
        n, K = self.n, self.K
        per = 2 if self.with_val else 1
        base = (self.gathered if self.sharded else self.rec).data_ptr()
        ptrs = (ctypes.c_void_p(base), ctypes.c_void_p(base + 8 * per * K * n))
        shard = (n, K * self.rbytes) if self.sharded else (0, 0)
        return ptrs + (8 * per * n, 4 * per * n) + shard

    def population(self):
        """Contiguous (train_f f64[P], train_t i32[P], val_f, val_t) of the whole
        population (torch ops; for the separate tell/val-update entry points)."""
        n, P = self.n, self.P
        if not self.sharded:
            return self.train[0][:P], self.train[1][:P], self.val[0][:P], self.val[1][:P]
        g = self.gathered.view(self.world, record_bytes(n))
        f = g[:, :16 * n].contiguous().view(torch.float64).view(self.world, 2 * n)
        t = g[:, 16 * n:].contiguous().view(torch.int32).view(self.world, 2 * n)
        return (f[:, :n].reshape(-1)[:P].contiguous(), t[:, :n].reshape(-1)[:P].contiguous(),
                f[:, n:].reshape(-1)[:P].contiguous(), t[:, n:].reshape(-1)[:P].contiguous())


def read_gathered(buf: np.ndarray, i: int, n: int, field: str):
    """Host mirror of the kernel's shard addressing (tests)."""
    off = element_offset(i, n, field)
    dt = np.float64 if field.endswith("_f") else np.int32
    return buf[off:off + np.dtype(dt).itemsize].view(dt)[0]
