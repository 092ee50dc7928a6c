"""Population fitness engine: drop-in for Env/drl_engine.py.

``evaluate_individual``  -- same signature/return as drl_engine.py:9-67.
``evaluate_population``  -- the batched form of ``pool.starmap(evaluate_individual,
                            zip(mm_pop, adv_pop))`` (drl_engine.py:104-115).
``DRLEngine``            -- same constructor / ``train`` signature and results as
                            drl_engine.py:69-178, with the generation loop
                            (ask -> rollout -> tell -> validation -> sigma decay)
                            resident on the GPU.

Every rollout runs in libsgmm.so (HIP, gfx950); without a GPU these functions
raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import AskedPopulation, GAHistory, GAState, check, ptr, stream_ptr
from .model import NeuroEvolution, TradingPolicy, genome_size, genome_to_state_dict, hidden_from_genome
from .rollout import EnvConfig, EpisodeBatch, RolloutEngine, TickStore, params_tensor
from .shard import FitnessRecords, shard_bounds, shard_capacity  # noqa: F401 (re-exported)

ADV_GENOME = genome_size(32)  # adversary evolver masters are TradingPolicy() genomes (model.py:63)

_engines: dict = {}
_bundle_cache: "OrderedDict[bytes, TickStore]" = OrderedDict()


def _engine(device=None) -> RolloutEngine:
    dev = torch.device(device or "cuda")
    if dev not in _engines:
        _engines[dev] = RolloutEngine(dev)
    return _engines[dev]


def _bundle_key(bundles, train_stats) -> bytes:
    h = hashlib.blake2b(digest_size=16)
    for b in bundles:
        for a in b:
            a = np.ascontiguousarray(a)
            h.update(str(a.dtype).encode())
            h.update(a.tobytes())
    for k in ("s1_m", "s1_s", "s2_m", "s2_s"):
        v = train_stats[k]
        h.update(f"{k}:{type(v).__name__}:{float(v).hex()}".encode())
    return h.digest()


def device_ticks(bundles, train_stats, device=None) -> TickStore:
    """Upload (and cache) bundles as one SoA TickStore; segment i = bundles[i]."""
    key = _bundle_key(bundles, train_stats) + str(device).encode()
    ts = _bundle_cache.get(key)
    if ts is None:
        ts = TickStore()
        for b in bundles:
            ts.add(b, train_stats)
        ts.to(torch.device(device or "cuda"))
        _bundle_cache[key] = ts
        while len(_bundle_cache) > 8:
            _bundle_cache.popitem(last=False)
    else:
        _bundle_cache.move_to_end(key)
    return ts


def _stack(pop, n_params, device):
    if torch.is_tensor(pop):
        t = pop.reshape(-1, n_params)
    else:
        t = torch.stack([torch.as_tensor(w, dtype=torch.float32).reshape(-1) for w in pop])
    return t.to(device=device, dtype=torch.float32).contiguous()


def evaluate_population(mm_pop, adv_pop, bundle, phi, tick_size, fee_rate, train_stats,
                        use_arl=False, device=None):
    """Fitness of every (mm, adv) pair on one bundle: returns (f64[P], i32[P]).

    ``adv_pop`` may be None or contain None entries (no adversary for that pair),
    matching ``adv_weights is not None`` in drl_engine.py:16."""
    eng = _engine(device)
    dev = eng.device
    n_mm = len(mm_pop)
    G = (mm_pop.shape[1] if torch.is_tensor(mm_pop) else len(mm_pop[0]))
    H = hidden_from_genome(int(G))
    mm = _stack(mm_pop, G, dev)
    ticks = device_ticks([bundle], train_stats, dev)
    off, T = ticks.segments[0]
    adv = None
    adv_idx = None
    if use_arl and adv_pop is not None and any(a is not None for a in adv_pop):
        rows = [a if a is not None else torch.zeros(ADV_GENOME) for a in adv_pop]
        Ga = max(len(torch.as_tensor(r).reshape(-1)) for r in rows)
        adv = torch.zeros((len(rows), Ga), dtype=torch.float32)
        for i, r in enumerate(rows):
            r = torch.as_tensor(r, dtype=torch.float32).reshape(-1)
            adv[i, :len(r)] = r
        adv = adv.to(dev)
        adv_idx = np.array([i if a is not None else -1 for i, a in enumerate(adv_pop)], np.int32)
    eps = EpisodeBatch(genome=np.arange(n_mm), tick_off=np.full(n_mm, off), length=np.full(n_mm, T),
                       param=np.zeros(n_mm), adv=adv_idx).to(dev)
    params = params_tensor([EnvConfig(phi=phi, tick_size=tick_size, fee_rate=fee_rate)], dev)
    fit, trd = eng.fitness(ticks, eps, params, mm, H, adv)
    return fit.cpu().numpy(), trd.cpu().numpy()


def evaluate_individual(mm_weights, adv_weights, bundle, phi, tick_size, fee_rate, train_stats,
                        use_arl=False):
    """One episode (drl_engine.py:9-67) on the GPU: returns (total_reward, trades)."""
    fit, trd = evaluate_population([mm_weights], [adv_weights], bundle, phi, tick_size, fee_rate,
                                   train_stats, use_arl=use_arl)
    return np.float64(fit[0]), int(trd[0])


def _dist_info(dist):
    """(group, rank, world, group_active): group_active is False for one
    process -- dist=False, or no process group initialised -- even when a
    default group exists, so the session never touches that group."""
    if dist is False:
        return None, 0, 1, False
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        g = dist if dist not in (None, True) else None
        return g, torch.distributed.get_rank(g), torch.distributed.get_world_size(g), True
    return None, 0, 1, False


class DRLEngine:
    """Neuroevolution trainer (drl_engine.py:69-178), generation loop on device.

    Reference-compatible arguments; keyword-only extras:
      hidden_dim  -- TradingPolicy hidden width (reference: 32).
      rng         -- "device": populations from a counter-based Philox stream on
                     the GPU (fast, reproducible from ``seed``, identical on every
                     rank); "torch": the reference's torch CPU generator, so a run
                     under torch.manual_seed reproduces the reference's trajectory.
      seed        -- device RNG seed (default: drawn from the torch generator).
      val_mode    -- "fused": validate every individual in the training launch and
                     pick the best's value (removes a serial episode per generation);
                     "best": validate only the best after tell (reference order);
                     "auto": best from BEST_VAL_MIN_SHARD (256) individuals per
                     population shard, fused below.
      honor_sigma -- the reference ignores DRLEngine(sigma=...) (NeuroEvolution keeps
                     its 0.05 default, drl_engine.py:77); True uses it.
      sync_every  -- generations between host synchronisations (log lines and
                     checkpoint writes are emitted at these points, in order).
      dist        -- torch.distributed group (None = default if initialised,
                     False = single process): the population is sharded over ranks
                     and fitness is all-gathered once per generation.
      use_graph   -- capture generations in HIP graphs and replay them (rng="device");
                     with several ranks on RCCL the all-gather is captured too.
      exchange    -- "auto": shard + all-gather only with several ranks; "always":
                     take the sharded path (asked rollout, all-gather, GA step) on
                     one process too -- the multi-GPU path rehearsed on one GPU.
      walk_feedback -- True: the session owns a device walk order that the library
                     rewrites after each training launch (sgmm_populations::walk_order:
                     the lightest populations are walked whole next generation);
                     scheduling only, results do not depend on it.
    """

    def __init__(self, pop_size=50, sigma=0.05, phi=0.01, tick_size=0.01, fee_rate=0.0,
                 use_arl=False, save_dir="checkpoints/drl", *, hidden_dim=32, rng="device",
                 seed=None, val_mode="auto", honor_sigma=False, sync_every=10, dist=None,
                 device=None, verbose=True, patience=15, decay=0.5, use_graph=True, exchange="auto",
                 walk_feedback=True):
        self.phi = phi
        self.tick_size = tick_size
        self.fee_rate = fee_rate
        self.save_dir = save_dir
        os.makedirs(self.save_dir, exist_ok=True)
        self.use_arl = use_arl
        self.pop_size = int(pop_size)
        self.hidden_dim = int(hidden_dim)
        self.mm_evolver = NeuroEvolution(population_size=pop_size, hidden_dim=self.hidden_dim)
        if honor_sigma:
            self.mm_evolver.sigma = sigma
        if use_arl:
            self.adv_evolver = NeuroEvolution(population_size=pop_size)
            if honor_sigma:
                self.adv_evolver.sigma = sigma
        if rng not in ("device", "torch"):
            raise ValueError("rng must be 'device' or 'torch'")
        self.rng = rng
        if seed is not None:
            self.seed = int(seed)
        else:  # rng="torch" must not draw extra numbers from the reference stream
            self.seed = int(torch.randint(0, 2**62, (1,)).item()) if rng == "device" else 0
        self.val_mode = val_mode
        self.sync_every = max(1, int(sync_every))
        self.dist = dist
        self.device = device
        self.verbose = verbose
        self.patience = int(patience)
        self.decay = float(decay)
        self.use_graph = use_graph
        if exchange not in ("auto", "always"):
            raise ValueError("exchange must be 'auto' or 'always'")
        self.exchange = exchange
        self.walk_feedback = bool(walk_feedback)
        self.timing = {}

    def _log(self, msg):
        if self.verbose:
            print(msg)
            sys.stdout.flush()

    def session(self, train_bundle, val_bundle, train_stats, generations=100, output_prefix="agent"):
        """Device-resident training session: step(gen) enqueues one generation."""
        return TrainingSession(self, train_bundle, val_bundle, train_stats, generations, output_prefix)

    def train(self, train_bundle, val_bundle, train_stats, generations=100, output_prefix="agent"):
        sess = self.session(train_bundle, val_bundle, train_stats, generations, output_prefix)
        for gen in range(0, generations, self.sync_every):
            n = min(self.sync_every, generations - gen)
            sess.steps(gen, n)
            if n == self.sync_every:
                sess.flush(gen + n)
        return sess.finish()


class _GraphedGenerations:
    """Generation replay shared by TrainingSession and MultiSession.

    A generation is _rollout, _exchange, _boundary (the last two no-ops on one
    unsharded process).  With use_graph it is captured once and replayed; when
    the exchange is capturable -- one process, or RCCL (nccl backend) -- the
    whole generation, all-gather included, is ONE graph, and batches of
    GRAPH_BATCH generations are captured into one graph as well, so several
    ranks also run one host launch per batch.  Otherwise (gloo: the gather is
    staged through host memory) the rollout and the GA step are two graphs
    around an eager all-gather."""

    # generations per captured multi-generation graph
    GRAPH_BATCH = 16

    def _gen(self):
        self._rollout()
        self._exchange()
        self._boundary()

    def _collective_capturable(self) -> bool:
        if not self.sharded:
            return True
        import torch.distributed as tdist
        if not (self.group_active and tdist.is_available() and tdist.is_initialized()):
            return True  # one process (no group, or dist=False): the gather is a device copy
        return tdist.get_backend(self.group) == "nccl"

    def capture(self):
        """Record (without running) the generation graph(s) and the batch graph."""
        if not self.use_graph:
            return
        if self.graphs is None:
            if self._collective_capturable():
                try:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self._gen()
                    self.graphs, self.full_graph = [g], True
                except Exception as ex:  # an RCCL build that cannot capture: eager exchange
                    if not self.sharded:
                        raise
                    self.full_graph = False
                    self.capture_error = repr(ex)
            if not self.full_graph:
                self.graphs = []
                for fn in (self._rollout, self._boundary):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        fn()
                    self.graphs.append(g)
        if self.full_graph and self.graph_batch > 1 and self.batch_graph is None:
            # batches of graph_batch, graph_batch / 2, ..., 2 generations: any
            # generation count replays as at most log2(graph_batch) + 1 graphs,
            # never as a train of single-generation replays paced by the host
            self.batch_graphs = {}
            B = self.graph_batch
            while B > 1:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(B):
                        self._gen()
                self.batch_graphs[B] = g
                B //= 2
            self.batch_graph = self.batch_graphs[self.graph_batch]

    def step(self, gen: int):
        """Enqueue generation ``gen`` (drl_engine.py:92-171) on the current stream."""
        if not self.use_graph:
            self._gen()
            return
        self.capture()
        if self.full_graph:
            self.graphs[0].replay()
        else:
            self.graphs[0].replay()
            self._exchange()
            self.graphs[1].replay()

    def steps(self, gen0: int, n: int):
        """Enqueue generations gen0 .. gen0 + n - 1 (same as n step() calls):
        whole batches replay the batch graph (one host launch per batch; the
        host-side launch, not the GPU, paced single-generation replays)."""
        if self.use_graph:
            self.capture()
        if not self.use_graph or not self.full_graph:
            for g in range(gen0, gen0 + n):
                self.step(g)
            return
        done = 0
        for B in sorted(self.batch_graphs, reverse=True):
            while n - done >= B:
                self.batch_graphs[B].replay()
                done += B
        for g in range(gen0 + done, gen0 + n):
            self.step(g)


class TrainingSession(_GraphedGenerations):
    """One DRLEngine.train run, resident on the GPU (drl_engine.py:83-178).

    Per generation (step): ask the shard's genomes -> roll the shard out (train,
    plus validation when fused) -> all-gather fitness over ranks -> tell both
    evolvers -> validation bookkeeping (checkpoint slot, sigma decay, history).
    Nothing in step() waits for the device; flush() brings history rows to the
    host, prints the reference's log lines in order and writes the checkpoint."""

    def __init__(self, eng: DRLEngine, train_bundle, val_bundle, train_stats, generations, output_prefix):
        _lib.require_gpu()
        self.e = eng
        # a session owns its workspace: a captured graph keeps raw pointers to it
        self.roll = RolloutEngine(eng.device or "cuda")
        dev = self.dev = self.roll.device
        self.L = self.roll.L
        self.group, self.rank, self.world, self.group_active = _dist_info(eng.dist)
        self.sharded = self.world > 1 or eng.exchange == "always"
        P, H = eng.pop_size, eng.hidden_dim
        self.P, self.H, self.G = P, H, genome_size(H)
        G = self.G
        self.i0, self.i1 = shard_bounds(P, self.rank, self.world)
        n_loc = self.n_loc = self.i1 - self.i0
        n_cap = self.n_cap = shard_capacity(P, self.world)  # record slots per rank
        arl = self.arl = eng.use_arl
        self.fused = not _best_validation(eng.val_mode, n_cap)
        self.torch_rng = eng.rng == "torch"
        # device RNG, validation of the best: the populations path with K = 1
        # (asked rollout + tell in its tail, then the new master's validation)
        self.best_step = not self.torch_rng and not self.fused and G_ok(H)
        self.generations = int(generations)
        # (rng="torch" with world > 1: every rank draws the identical full
        # population from its identically seeded generator)
        self.ticks = device_ticks([train_bundle, val_bundle], train_stats, dev)
        (tr_off, self.T_tr), (va_off, self.T_va) = self.ticks.segments
        self.params = params_tensor([EnvConfig(phi=eng.phi, tick_size=eng.tick_size,
                                               fee_rate=eng.fee_rate)], dev)
        # episode slots follow the record layout: n_cap per phase, the shard's
        # n_loc individuals first, then zero-length pads (never read back)
        pad = n_cap - n_loc

        def phase(off, T):
            return (np.concatenate([np.arange(n_loc), np.zeros(pad, np.int64)]),
                    np.full(n_cap, off), np.concatenate([np.full(n_loc, T), np.zeros(pad, np.int64)]))

        g_tr, o_tr, l_tr = phase(tr_off, self.T_tr)
        g_va, o_va, l_va = phase(va_off, self.T_va)
        self.rec = FitnessRecords(P, self.world, dev, gather=self.sharded, with_val=not self.best_step,
                                  group_active=self.group_active)
        if self.fused:  # one launch: training + validation episodes of the shard
            adv = np.concatenate([g_tr, np.full(n_cap, -1)]) if arl else None  # validation: no adversary
            self.train_eps = EpisodeBatch(np.concatenate([g_tr, g_va]), np.concatenate([o_tr, o_va]),
                                          np.concatenate([l_tr, l_va]), np.zeros(2 * n_cap), adv=adv).to(dev)
            self.val_eps = None
            self.out, self.vout = self.rec.both, None
        else:
            self.train_eps = EpisodeBatch(g_tr, o_tr, l_tr, np.zeros(n_cap),
                                          adv=g_tr if arl else None).to(dev)
            self.out = self.rec.train
            # validation of the best only (reference order)
            self.val_eps = EpisodeBatch(np.zeros(1), np.full(1, va_off), np.full(1, self.T_va),
                                        np.zeros(1)).to(dev)
            self.vout = (torch.empty(1, dtype=torch.float64, device=dev),
                         torch.empty(1, dtype=torch.int32, device=dev))
        f32 = dict(dtype=torch.float32, device=dev)
        # population rows: the full population when the host draws it (torch
        # RNG), else the shard's capacity (pads point at row 0, which exists)
        n_rows = P if self.torch_rng else max(n_cap, 1)
        if not self.torch_rng and G <= 4096:
            n_rows = 1  # asked population: generated inside the rollout (placeholder row)
        self.pop = torch.empty((n_rows, G), **f32)
        lo = min(self.i0, P - 1)
        self.pop_loc = self.pop[lo:lo + max(n_cap, 1)] if self.torch_rng else self.pop
        self.adv_pop = torch.empty((n_rows, ADV_GENOME), **f32) if arl else None
        self.adv_loc = (self.adv_pop[lo:lo + max(n_cap, 1)] if self.torch_rng else self.adv_pop) if arl else None
        self.master = eng.mm_evolver.master_policy.get_weights().to(**f32)
        self.master_adv = eng.adv_evolver.master_policy.get_weights().to(**f32) if arl else None
        self.best_master = torch.zeros(G, **f32)
        self.state = torch.zeros(HIST_STATE_SIZES[0], dtype=torch.uint8, device=dev)
        self.hist = torch.zeros((self.generations, HIST_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        if arl and eng.adv_evolver.sigma != eng.mm_evolver.sigma:
            raise ValueError("mm and adversary sigma must start equal (one device state holds both)")
        check(self.L.sgmm_ga_state_init(ptr(self.state), float(eng.mm_evolver.sigma), eng.patience,
                                        eng.decay, stream_ptr()), "sgmm_ga_state_init")
        # device RNG + fused validation: the population is never materialized --
        # the rollout kernels generate each individual's genome from the master
        # and the GA state, and the GA step runs in the rollout's last workgroup
        # (one process) or after the all-gather (several ranks)
        self.fast_step = (not self.torch_rng and self.fused and G <= 4096 and ADV_GENOME <= 4096)
        self.asked = AskedPopulation(self.state.data_ptr(), self.master.data_ptr(),
                                     self.master_adv.data_ptr() if arl else None, eng.seed, self.i0, 0)
        self.seeds = torch.tensor([int(eng.seed)], dtype=torch.int64).to(dev)
        # the frontier kernel's walk order, rewritten on the device by the walk-order
        # feedback (sgmm_populations::walk_order); train_eps stays read-only
        self.walk_order = self.train_eps.dev["order"].clone()
        self.pops = _lib.Populations(1, P, H, self.generations, self.state.data_ptr(), self.master.data_ptr(),
                                     self.master_adv.data_ptr() if arl else None, self.best_master.data_ptr(),
                                     self.seeds.data_ptr(), self.hist.data_ptr(),
                                     self.walk_order.data_ptr() if eng.walk_feedback else None)
        # one generation = fixed launches -> replayable HIP graphs: the whole
        # generation on one rank; with several ranks the rollout and the boundary
        # are captured separately around the (eager) all-gather
        self.use_graph = bool(eng.use_graph) and not self.torch_rng
        self.graphs, self.batch_graph, self.batch_graphs, self.full_graph = None, None, {}, False
        self.graph_batch = max(1, min(self.GRAPH_BATCH, eng.sync_every))
        self.roll.reserve(self.train_eps, arl)
        if self.val_eps is not None:
            self.roll.reserve(self.val_eps, False)
        self.best_path = os.path.join(eng.save_dir, f"{output_prefix}_best_val_{eng.phi}.pth")
        self.saved_any = False
        self.emitted = 0
        self.history = {"gen": [], "train_f": [], "val_f": [], "train_trades": [], "val_trades": []}
        self.ev0 = torch.cuda.Event(enable_timing=True)
        self.ev1 = torch.cuda.Event(enable_timing=True)
        self.ev0.record()

    def _ask(self):
        """ask() of the shard (models/model.py:65-71) from the device master/sigma."""
        e, L, s, G = self.e, self.L, stream_ptr(), self.G
        check(L.sgmm_ga_ask(ptr(self.master), G, ptr(self.state), 0, e.seed, self.i0, self.n_loc,
                            ptr(self.pop), G, s), "sgmm_ga_ask")
        if self.arl:
            check(L.sgmm_ga_ask(ptr(self.master_adv), ADV_GENOME, ptr(self.state), 1, e.seed, self.i0,
                                self.n_loc, ptr(self.adv_pop), ADV_GENOME, s), "sgmm_ga_ask(adv)")

    def _rollout(self):
        """ask (host draw / device kernel / generated in-kernel) + the shard's
        rollouts (drl_engine.py:104-115, plus the fused validation episodes);
        with one process and the asked population the whole generation,
        including the GA step, is this one call."""
        P = self.P
        L, s = self.L, stream_ptr()
        if self.best_step:
            tk, ep = self.ticks.struct(), self.train_eps.struct()
            ws = self.roll.workspace(self.train_eps, self.arl)
            f, t = self.out
            if not self.sharded:
                vep = self.val_eps.struct()
                vf, vt = self.vout
                check(L.sgmm_generation_multi_best(ctypes.byref(tk), ctypes.byref(ep), ctypes.byref(vep),
                                                   ptr(self.params), ctypes.byref(self.pops), ptr(f), ptr(t),
                                                   ptr(vf), ptr(vt), ptr(ws), ws.numel(), s),
                      "sgmm_generation_multi_best")
            else:
                check(L.sgmm_rollout_fitness_asked(ctypes.byref(tk), ctypes.byref(ep), ptr(self.params),
                                                   ctypes.byref(self.asked), self.H, ptr(f), ptr(t), ptr(ws),
                                                   ws.numel(), s), "sgmm_rollout_fitness_asked")
            return
        if self.fast_step:
            tk, ep = self.ticks.struct(), self.train_eps.struct()
            ws = self.roll.workspace(self.train_eps, self.arl)
            f, t = self.out
            if not self.sharded:
                check(L.sgmm_generation(ctypes.byref(tk), ctypes.byref(ep), ptr(self.params), ptr(self.state),
                                        ptr(self.master), ptr(self.master_adv) if self.arl else None,
                                        ptr(self.best_master), self.H, self.e.seed, P, ptr(f), ptr(t),
                                        ptr(self.hist), self.generations, ptr(ws), ws.numel(), s),
                      "sgmm_generation")
            else:
                check(L.sgmm_rollout_fitness_asked(ctypes.byref(tk), ctypes.byref(ep), ptr(self.params),
                                                   ctypes.byref(self.asked), self.H, ptr(f), ptr(t), ptr(ws),
                                                   ws.numel(), s), "sgmm_rollout_fitness_asked")
            return
        if self.torch_rng:
            st_now = self.state.cpu().numpy().view(STATE_DTYPE)[0]
            self.pop.copy_(_host_ask(self.master, float(st_now["sigma_mm"]), P))
            if self.arl:
                self.adv_pop.copy_(_host_ask(self.master_adv, float(st_now["sigma_adv"]), P))
        else:
            self._ask()
        self.roll.fitness(self.ticks, self.train_eps, self.params, self.pop_loc, self.H, self.adv_loc,
                          out=self.out)

    def _exchange(self):
        """The generation's one collective: all-gather the per-rank records."""
        if self.sharded:
            self.rec.all_gather(self.group)

    def _boundary(self):
        """tell both evolvers, validation bookkeeping, sigma decay (after the
        exchange; a no-op when the generation call already did it)."""
        e, L, s = self.e, self.L, stream_ptr()
        P, G = self.P, self.G
        arl = self.arl
        if self.best_step:
            if self.sharded:  # every rank: tell on the gathered records, then validate the new master
                check(L.sgmm_ga_tell_multi(ctypes.byref(self.pops), *self.rec.tell_args(), s), "sgmm_ga_tell_multi")
                tk, vep = self.ticks.struct(), self.val_eps.struct()
                ws = self.roll.workspace(self.val_eps, False)
                vf, vt = self.vout
                check(L.sgmm_validate_multi(ctypes.byref(tk), ctypes.byref(vep), ptr(self.params),
                                            ctypes.byref(self.pops), ptr(vf), ptr(vt), ptr(ws), ws.numel(), s),
                      "sgmm_validate_multi")
            return
        if self.fast_step:
            if self.sharded:
                check(L.sgmm_ga_step(ptr(self.state), *self.rec.step_args(),
                                     ptr(self.master), ptr(self.master_adv) if arl else None,
                                     ptr(self.best_master), G, ADV_GENOME if arl else 0, e.seed,
                                     ptr(self.hist), self.generations, None, None, 0, 0, s),
                      "sgmm_ga_step")
            return
        tr_f, tr_t, va_f, va_t = self.rec.population()
        # tell both evolvers (model.py:73-76, drl_engine.py:119-125)
        check(L.sgmm_ga_tell(ptr(self.state), ptr(tr_f), ptr(tr_t), P, ptr(self.master),
                             ptr(self.pop) if self.torch_rng else None, G,
                             ptr(self.master_adv) if arl else None,
                             ptr(self.adv_pop) if (arl and self.torch_rng) else None, ADV_GENOME, G,
                             ADV_GENOME if arl else 0, e.seed, ptr(self.hist), self.generations, s),
              "sgmm_ga_tell")
        # validation of the best (drl_engine.py:129-171)
        if not self.fused:
            self.roll.fitness(self.ticks, self.val_eps, self.params, self.master.view(1, G), self.H, None,
                              out=self.vout)
            va_f, va_t = self.vout
        check(L.sgmm_ga_val_update(ptr(self.state), ptr(va_f), ptr(va_t), 1 if self.fused else 0,
                                   ptr(self.master), ptr(self.best_master), G, ptr(self.hist),
                                   self.generations, s), "sgmm_ga_val_update")
        if self.torch_rng:
            TradingPolicy()  # the reference's validation builds a TradingPolicy() (RNG draw)

    def flush(self, upto: int):
        """History rows [emitted, upto) to the host: log lines, checkpoint."""
        if upto <= self.emitted:
            return
        e = self.e
        rows = self.hist[self.emitted:upto].cpu().numpy().view(HIST_DTYPE).reshape(-1)
        improved_any = False
        for k, r in enumerate(rows):
            g = self.emitted + k
            imp = bool(r["flags"] & 1)
            improved_any |= imp
            if r["flags"] & 2:
                e._log(f">>> Sigma decayed to {r['sigma_after']:.4f} due to no improvement")
            self.history["gen"].append(g)
            self.history["train_f"].append(np.float64(r["train_f"]))
            self.history["val_f"].append(np.float64(r["val_f"]))
            self.history["train_trades"].append(int(r["train_trades"]))
            self.history["val_trades"].append(int(r["val_trades"]))
            if g % 5 == 0:
                tag = "ARL:ON" if self.arl else "ARL:OFF"
                e._log(f"Gen {g:03d} | {tag} | Best Train: {r['train_f']:.2f} | "
                       f"Val: {r['val_f']:.2f}{'*' if imp else ''}")
        if improved_any and self.rank == 0:
            torch.save(genome_to_state_dict(self.best_master, self.H), self.best_path)
        self.saved_any |= improved_any
        self.emitted = upto

    def finish(self):
        """Flush, copy the evolver state back, reload the best-validation weights
        (drl_engine.py:174-178); returns (master_policy, history)."""
        e = self.e
        self.ev1.record()
        self.flush(self.generations)
        torch.cuda.synchronize()
        e.timing = {"generations": self.generations, "ms": self.ev0.elapsed_time(self.ev1),
                    "env_steps": self.generations * self.P * self.T_tr}
        st = self.state.cpu().numpy().view(STATE_DTYPE)[0]
        e.mm_evolver.sigma = float(st["sigma_mm"])
        e.mm_evolver.master_policy.set_weights(self.master.cpu())
        if self.arl:
            e.adv_evolver.sigma = float(st["sigma_adv"])
            e.adv_evolver.master_policy.set_weights(self.master_adv.cpu())
        if self.saved_any:
            e.mm_evolver.master_policy.load_state_dict(genome_to_state_dict(self.best_master, self.H))
        elif os.path.exists(self.best_path):
            e.mm_evolver.master_policy.load_state_dict(torch.load(self.best_path, weights_only=True))
        return e.mm_evolver.master_policy, self.history


class MultiDRLEngine:
    """K independent DRLEngine.train runs advanced together on the GPU.

    The reference trains one GA per inventory penalty phi (the lambda sweep:
    run_agent_training_pipeline per PHI, main.py:39-45 ->
    agent_trainer.py:136-137; checkpoints/688981/agent_best_val_{phi}.pth) and
    one per asset (agent_trainer.py:168-173).  Here the K runs share every
    generation's launches: population k keeps its own master, sigma schedule,
    no-improvement counter, best validation reward, history, checkpoint path
    ``{save_dir}/{prefix}_best_val_{phi}.pth`` and Philox key, so its results
    are bit-identical to ``engines[k].train(...)`` run alone.

    ``engines`` are configured DRLEngine objects (same pop_size, hidden_dim and
    use_arl; rng="device"); ``MultiDRLEngine.sweep(phis, ...)`` builds one per
    phi.  ``train`` takes one bundle (shared) or a list of K bundles (one per
    population, e.g. per asset), likewise train_stats, and returns the list of
    K (master_policy, history) results in engine order.
    """

    def __init__(self, engines):
        self.engines = list(engines)
        if not self.engines:
            raise ValueError("MultiDRLEngine needs at least one DRLEngine")
        e0 = self.engines[0]
        for e in self.engines[1:]:
            if (e.pop_size, e.hidden_dim, e.use_arl) != (e0.pop_size, e0.hidden_dim, e0.use_arl):
                raise ValueError("populations of one MultiDRLEngine share pop_size, hidden_dim and use_arl")

    @classmethod
    def sweep(cls, phis, pop_size=50, sigma=0.05, tick_size=0.01, fee_rate=0.0, use_arl=False,
              save_dir="checkpoints/drl", *, seeds=None, **kw):
        """One DRLEngine per phi (the lambda sweep), constructed in phi order."""
        engines = [DRLEngine(pop_size, sigma, phi, tick_size, fee_rate, use_arl, save_dir,
                             seed=None if seeds is None else seeds[k], **kw)
                   for k, phi in enumerate(phis)]
        return cls(engines)

    @property
    def fused_path(self) -> bool:
        """All populations on the shared device path (else: one after another)."""
        return all(e.rng == "device" and genome_size(e.hidden_dim) <= 4096 for e in self.engines) and \
            len({e.val_mode for e in self.engines}) == 1

    def session(self, train_bundles, val_bundles, train_stats, generations=100, output_prefix="agent"):
        return MultiSession(self, train_bundles, val_bundles, train_stats, generations, output_prefix)

    def train(self, train_bundles, val_bundles, train_stats, generations=100, output_prefix="agent"):
        K = len(self.engines)
        tr, va, st = (_per_pop(x, K) for x in (train_bundles, val_bundles, train_stats))
        if not self.fused_path:  # reference order: one DRLEngine.train after another
            return [e.train(tr[k], va[k], st[k], generations, output_prefix) for k, e in enumerate(self.engines)]
        sess = self.session(tr, va, st, generations, output_prefix)
        every = self.engines[0].sync_every
        for gen in range(0, generations, every):
            n = min(every, generations - gen)
            sess.steps(gen, n)
            if n == every:
                sess.flush(gen + n)
        return sess.finish()


def _per_pop(x, K):
    """One bundle / stats dict for all populations, or a list of K of them."""
    if isinstance(x, dict) or (isinstance(x, tuple) and len(x) == 7 and not isinstance(x[0], (tuple, list))):
        return [x] * K
    x = list(x)
    if len(x) != K:
        raise ValueError(f"expected {K} per-population items, got {len(x)}")
    return x


class MultiSession(_GraphedGenerations):
    """K DRLEngine.train runs resident on the GPU, one launch pair per
    generation for all of them (sgmm_generation_multi), or -- with several
    ranks -- the asked rollout of every population's shard, one all-gather of
    the K records and one K-workgroup GA step (sgmm_ga_step_multi)."""

    def __init__(self, meng: MultiDRLEngine, train_bundles, val_bundles, train_stats, generations,
                 output_prefix):
        _lib.require_gpu()
        engs = self.engs = meng.engines
        e0 = engs[0]
        K = self.K = len(engs)
        tr, va, sts = (_per_pop(x, K) for x in (train_bundles, val_bundles, train_stats))
        self.roll = RolloutEngine(e0.device or "cuda")
        dev = self.dev = self.roll.device
        self.L = self.roll.L
        self.group, self.rank, self.world, self.group_active = _dist_info(e0.dist)
        self.sharded = self.world > 1 or e0.exchange == "always"
        P, H = self.P, self.H = e0.pop_size, e0.hidden_dim
        G = self.G = genome_size(H)
        self.i0, self.i1 = shard_bounds(P, self.rank, self.world)
        n_loc = self.n_loc = self.i1 - self.i0
        n = self.n_cap = shard_capacity(P, self.world)
        arl = self.arl = e0.use_arl
        self.generations = int(generations)
        # tick columns: each distinct (bundle, stats) once
        self.ticks = TickStore()
        seg_of = {}

        def seg(b, s):
            key = (id(b), id(s))
            if key not in seg_of:
                seg_of[key] = self.ticks.segments[self.ticks.add(b, s)]
            return seg_of[key]

        segs = [(seg(tr[k], sts[k]), seg(va[k], sts[k])) for k in range(K)]
        self.ticks.to(dev)
        self.T_tr = [s[0][1] for s in segs]
        self.params = params_tensor([EnvConfig(phi=e.phi, tick_size=e.tick_size, fee_rate=e.fee_rate)
                                     for e in engs], dev)
        # validation: "fused" validates every individual inside the training
        # launch (one launch pair per generation); "best" validates only each
        # population's new master after the tell (the reference's order:
        # sgmm_generation_multi_best, four launches but K validation episodes
        # instead of K * P)
        self.best_val = _best_validation(e0.val_mode, n, K)
        # episodes: per population n training slots (then n validation slots
        # when fused) -- the shard's n_loc individuals first, zero-length pads after
        pad = n - n_loc
        g, off, ln, par, adv = [], [], [], [], []
        for k, ((to, T), (vo, Tv)) in enumerate(segs):
            phases = ((to, T, True),) if self.best_val else ((to, T, True), (vo, Tv, False))
            for o, L_, is_tr in phases:
                g.append(np.concatenate([np.arange(n_loc), np.zeros(pad, np.int64)]))
                off.append(np.full(n, o))
                ln.append(np.concatenate([np.full(n_loc, L_), np.zeros(pad, np.int64)]))
                par.append(np.full(n, k))
                adv.append(g[-1] if is_tr else np.full(n, -1))  # validation: no adversary
        self.eps = EpisodeBatch(np.concatenate(g), np.concatenate(off), np.concatenate(ln), np.concatenate(par),
                                adv=np.concatenate(adv) if arl else None).to(dev)
        # best: one validation episode per population, genome row k = master k
        self.val_eps = EpisodeBatch(np.arange(K), np.array([s[1][0] for s in segs]),
                                    np.array([s[1][1] for s in segs]), np.arange(K)).to(dev) \
            if self.best_val else None
        self.vout = (torch.zeros(K, dtype=torch.float64, device=dev),
                     torch.zeros(K, dtype=torch.int32, device=dev)) if self.best_val else None
        self.rec = FitnessRecords(P, self.world, dev, n_pop=K, gather=self.sharded, with_val=not self.best_val,
                                  group_active=self.group_active)
        f32 = dict(dtype=torch.float32, device=dev)
        self.masters = torch.stack([e.mm_evolver.master_policy.get_weights() for e in engs]).to(**f32).contiguous()
        self.masters_adv = torch.stack([e.adv_evolver.master_policy.get_weights() for e in engs]).to(**f32) \
            .contiguous() if arl else None
        self.best_masters = torch.zeros((K, G), **f32)
        self.states = torch.zeros((K, HIST_STATE_SIZES[0]), dtype=torch.uint8, device=dev)
        self.hist = torch.zeros((K, self.generations, HIST_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.seeds = torch.tensor([int(e.seed) for e in engs], dtype=torch.int64).to(dev)
        for k, e in enumerate(engs):
            if arl and e.adv_evolver.sigma != e.mm_evolver.sigma:
                raise ValueError("mm and adversary sigma must start equal (one device state holds both)")
            check(self.L.sgmm_ga_state_init(ctypes.c_void_p(self.states[k].data_ptr()), float(e.mm_evolver.sigma),
                                            e.patience, e.decay, stream_ptr()), "sgmm_ga_state_init")
        # the frontier kernel's walk order, rewritten on the device by the walk-order
        # feedback (sgmm_populations::walk_order); the episode batch stays read-only
        self.walk_order = self.eps.dev["order"].clone()
        self.pops = _lib.Populations(K, P, H, self.generations, self.states.data_ptr(), self.masters.data_ptr(),
                                     self.masters_adv.data_ptr() if arl else None, self.best_masters.data_ptr(),
                                     self.seeds.data_ptr(), self.hist.data_ptr(),
                                     self.walk_order.data_ptr() if e0.walk_feedback else None)
        self.use_graph = bool(e0.use_graph)
        self.graphs, self.batch_graph, self.batch_graphs, self.full_graph = None, None, {}, False
        self.graph_batch = max(1, min(self.GRAPH_BATCH, e0.sync_every))
        self.roll.reserve(self.eps, arl)
        if self.val_eps is not None:
            self.roll.reserve(self.val_eps, False)
        self.best_paths = [os.path.join(e.save_dir, f"{output_prefix}_best_val_{e.phi}.pth") for e in engs]
        self.saved_any = [False] * K
        self.emitted = 0
        self.history = [{"gen": [], "train_f": [], "val_f": [], "train_trades": [], "val_trades": []}
                        for _ in range(K)]

    # one generation: rollout (+ GA step in its tail on one process)
    def _rollout(self):
        tk, ep = self.ticks.struct(), self.eps.struct()
        ws = self.roll.workspace(self.eps, self.arl)
        f, t = self.rec.both
        if not self.sharded and self.best_val:
            vep = self.val_eps.struct()
            vf, vt = self.vout
            check(self.L.sgmm_generation_multi_best(ctypes.byref(tk), ctypes.byref(ep), ctypes.byref(vep),
                                                    ptr(self.params), ctypes.byref(self.pops), ptr(f), ptr(t),
                                                    ptr(vf), ptr(vt), ptr(ws), ws.numel(), stream_ptr()),
                  "sgmm_generation_multi_best")
        elif not self.sharded:
            check(self.L.sgmm_generation_multi(ctypes.byref(tk), ctypes.byref(ep), ptr(self.params),
                                               ctypes.byref(self.pops), ptr(f), ptr(t), ptr(ws), ws.numel(),
                                               stream_ptr()), "sgmm_generation_multi")
        else:
            per_pop = self.n_cap if self.best_val else 2 * self.n_cap
            check(self.L.sgmm_rollout_fitness_asked_multi(ctypes.byref(tk), ctypes.byref(ep), ptr(self.params),
                                                          ctypes.byref(self.pops), self.i0, per_pop,
                                                          ptr(f), ptr(t), ptr(ws), ws.numel(), stream_ptr()),
                  "sgmm_rollout_fitness_asked_multi")

    def _exchange(self):
        if self.sharded:
            self.rec.all_gather(self.group)

    def _boundary(self):
        if not self.sharded:
            return
        if self.best_val:  # every rank: tell on the gathered records, then validate the new masters
            check(self.L.sgmm_ga_tell_multi(ctypes.byref(self.pops), *self.rec.tell_args(), stream_ptr()),
                  "sgmm_ga_tell_multi")
            tk, vep = self.ticks.struct(), self.val_eps.struct()
            ws = self.roll.workspace(self.val_eps, False)
            vf, vt = self.vout
            check(self.L.sgmm_validate_multi(ctypes.byref(tk), ctypes.byref(vep), ptr(self.params),
                                             ctypes.byref(self.pops), ptr(vf), ptr(vt), ptr(ws), ws.numel(),
                                             stream_ptr()), "sgmm_validate_multi")
        else:
            check(self.L.sgmm_ga_step_multi(ctypes.byref(self.pops), *self.rec.multi_step_args(), stream_ptr()),
                  "sgmm_ga_step_multi")

    def flush(self, upto: int):
        """History rows [emitted, upto) of every population: the reference's log
        lines (prefixed with the population's phi), checkpoints."""
        if upto <= self.emitted:
            return
        rows_all = self.hist[:, self.emitted:upto].cpu().numpy()
        for k, e in enumerate(self.engs):
            rows = rows_all[k].reshape(-1).view(HIST_DTYPE)
            improved_any = False
            h = self.history[k]
            for j, r in enumerate(rows):
                g = self.emitted + j
                imp = bool(r["flags"] & 1)
                improved_any |= imp
                if r["flags"] & 2:
                    e._log(f"[phi={e.phi}] >>> Sigma decayed to {r['sigma_after']:.4f} due to no improvement")
                h["gen"].append(g)
                h["train_f"].append(np.float64(r["train_f"]))
                h["val_f"].append(np.float64(r["val_f"]))
                h["train_trades"].append(int(r["train_trades"]))
                h["val_trades"].append(int(r["val_trades"]))
                if g % 5 == 0:
                    tag = "ARL:ON" if self.arl else "ARL:OFF"
                    e._log(f"[phi={e.phi}] Gen {g:03d} | {tag} | Best Train: {r['train_f']:.2f} | "
                           f"Val: {r['val_f']:.2f}{'*' if imp else ''}")
            if improved_any and self.rank == 0:
                torch.save(genome_to_state_dict(self.best_masters[k], self.H), self.best_paths[k])
            self.saved_any[k] |= improved_any
        self.emitted = upto

    def finish(self):
        self.flush(self.generations)
        torch.cuda.synchronize()
        st = self.states.cpu().numpy().reshape(-1).view(STATE_DTYPE)
        out = []
        for k, e in enumerate(self.engs):
            e.mm_evolver.sigma = float(st[k]["sigma_mm"])
            e.mm_evolver.master_policy.set_weights(self.masters[k].cpu())
            if self.arl:
                e.adv_evolver.sigma = float(st[k]["sigma_adv"])
                e.adv_evolver.master_policy.set_weights(self.masters_adv[k].cpu())
            if self.saved_any[k]:
                e.mm_evolver.master_policy.load_state_dict(genome_to_state_dict(self.best_masters[k], self.H))
            elif os.path.exists(self.best_paths[k]):
                e.mm_evolver.master_policy.load_state_dict(torch.load(self.best_paths[k], weights_only=True))
            e.timing = {"generations": self.generations}
            out.append((e.mm_evolver.master_policy, self.history[k]))
        return out


# ---------------------------------------------------------------------- small helpers
# val_mode="auto": validate only the best (after the tell) from this many
# individuals per population shard; below it the fused launch's extra
# validation episodes cost less than the two extra launches
BEST_VAL_MIN_SHARD = 256


def G_ok(hidden: int) -> bool:
    """Genomes small enough for the device GA step (and the adversary's)."""
    return genome_size(hidden) <= 4096 and ADV_GENOME <= 4096


def _best_validation(val_mode: str, n_shard: int, n_pop: int = 1) -> bool:
    if val_mode not in ("auto", "fused", "best"):
        raise ValueError("val_mode must be 'auto', 'fused' or 'best'")
    return val_mode == "best" or (val_mode == "auto" and n_shard >= BEST_VAL_MIN_SHARD)


def ctypes_size(t):
    import ctypes
    return ctypes.sizeof(t)


def ctypes_offset_ptr(tensor, offset):
    import ctypes
    return ctypes.c_void_p(tensor.data_ptr() + int(offset))


HIST_DTYPE = np.dtype([("train_f", "<f8"), ("val_f", "<f8"), ("sigma_after", "<f8"),
                       ("train_trades", "<i4"), ("val_trades", "<i4"), ("best_idx", "<i4"),
                       ("flags", "<i4")])
STATE_DTYPE = np.dtype([("sigma_mm", "<f8"), ("sigma_adv", "<f8"), ("best_val", "<f8"),
                        ("last_train_f", "<f8"), ("last_val_f", "<f8"), ("no_improve", "<i4"),
                        ("best_idx", "<i4"), ("adv_best_idx", "<i4"), ("gen", "<i4"),
                        ("improved", "<i4"), ("decayed", "<i4"), ("patience", "<i4"),
                        ("arrivals", "<i4"), ("decay", "<f8")])
assert HIST_DTYPE.itemsize == ctypes_size(GAHistory) and STATE_DTYPE.itemsize == ctypes_size(GAState)
HIST_STATE_SIZES = (STATE_DTYPE.itemsize, HIST_DTYPE.itemsize)


def _host_ask(master_dev, sigma, P):
    """NeuroEvolution.ask on the torch CPU generator (reference stream), uploaded."""
    m = master_dev.cpu()
    return torch.stack([m + torch.randn_like(m) * sigma for _ in range(P)]).to(master_dev.device)
