/*
 * sgmm.h -- C ABI of the MI355X population-rollout library (libsgmm.so).
 *
 * Drop-in boundary for the hot path of the reference repository
 * (KAS-W/Deep-Reinforcement-Learning-Based-Signal-Gated-Market-Making).
 * The reference has no FFI: its boundary is a set of Python call signatures.
 * Each entry point below names the reference interface it replaces
 * (paths relative to the reference root); INTEGRATION.md shows the
 * Python (ctypes) binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - Every pointer argument is caller-owned DEVICE memory (hipMalloc / torch
 *     CUDA tensors) unless stated otherwise.  No entry point allocates, frees
 *     or synchronises in the hot calls: work is enqueued on `stream`
 *     (a hipStream_t, NULL = default stream) and the call returns.
 *   - Return value: 0 = success, < 0 = error; sgmm_last_error() (thread-local)
 *     describes the last failure.  Argument errors are detected before any
 *     work is enqueued.
 *   - Calls on distinct streams are thread-safe.
 *   - Numerics: prices/cash/reward float64 without FMA contraction (the
 *     reference's operation order, market_env.py:30-58); policy MLP float32
 *     with each dot product evaluated as the k-ordered fused chain starting at
 *     the bias; actions = rint(raw * act_scale) (round half to even, np.round).
 */
#ifndef SGMM_H
#define SGMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGMM_ABI_VERSION 5

enum {
    SGMM_OK = 0,
    SGMM_ERR_ARG = -1,       /* invalid argument (shape, pointer, range) */
    SGMM_ERR_HIP = -2,       /* HIP runtime error */
    SGMM_ERR_WORKSPACE = -3, /* workspace too small */
    SGMM_ERR_UNSUPPORTED = -4
};

/* Per-episode environment constants.
 * FTPEnv.__init__ (Env/market_env.py:8-15) plus the constants
 * evaluate_individual hard-codes (Env/drl_engine.py:39,48,64-65). */
typedef struct sgmm_env_params {
    double  phi;          /* inventory penalty lambda (market_env.py:10) */
    double  tick;         /* tick size (market_env.py:11) */
    double  fee;          /* fee rate (market_env.py:9) */
    double  idle_penalty; /* subtracted from fitness if no trade (drl_engine.py:64-65): 50.0 */
    int32_t i_max;        /* inventory cap (market_env.py:14): 2 */
    int32_t i_min;        /* inventory floor (market_env.py:15): -2 */
    float   act_scale;    /* MM action scale (drl_engine.py:39): 5.0 */
    float   adv_scale;    /* adversary action scale (drl_engine.py:48): 1.0 */
} sgmm_env_params;        /* 48 bytes */

/* The bundle (drl_engine.py:11) as structure-of-arrays device columns,
 * indexed by absolute tick index.  (sgmm_ticks and sgmm_episodes are HOST
 * structs whose members point to device memory.)  s1n/s2n are the normalised signals of
 * drl_engine.py:33-34 (host computes them once per bundle). */
typedef struct sgmm_ticks {
    const float  *s1n;
    const float  *s2n;
    const double *mid_next;
    const double *best_ask;
    const double *best_bid;
    const double *buy_max;
    const double *sell_min;
} sgmm_ticks;

/* A batch of episodes: episode e runs genome row genome[e] (and adversary
 * row adv[e], or -1 for none) over ticks [tick_off[e], tick_off[e]+len[e])
 * with params[param[e]].  step_off = exclusive prefix sum of len (it places
 * each episode's tables in the workspace); total_steps = sum of len.
 * Every episode of one call shares the inventory range [inv_min, inv_max]
 * (at most 8 inventory values; 0 must lie inside).  order (optional, may be
 * NULL) is a permutation of [0, n), longest episode first: the frontier
 * kernel (one wave per episode) starts the longest walks first so short ones
 * fill the tail; results are per episode and do not depend on it. */
typedef struct sgmm_episodes {
    int32_t        n;
    int32_t        max_len;
    int64_t        total_steps;
    int32_t        inv_min;   /* host copy of the (shared) i_min of params */
    int32_t        inv_max;   /* host copy of the (shared) i_max of params */
    const int32_t *genome;
    const int32_t *adv;       /* may be NULL (no adversary anywhere) */
    const int64_t *tick_off;
    const int32_t *len;
    const int64_t *step_off;
    const int32_t *param;
    const int32_t *order;     /* may be NULL: identity (ABI 2) */
} sgmm_episodes;

int         sgmm_abi_version(void);
const char *sgmm_last_error(void);

/* Batched FTPEnv.step over n independent environments.
 * Replaces Env/market_env.py:22-67 (FTPEnv.step).  inventory/cash are
 * updated in place; adv_action may be NULL (no adversary); reward / pnl /
 * inv_reward / fee_paid / fill_* outputs may individually be NULL.
 * params: device array, param_idx[n] (NULL = all use params[0]). */
int sgmm_env_step_batch(const sgmm_env_params *params, const int32_t *param_idx,
                        int32_t *inventory, double *cash,
                        const int32_t *action, const int32_t *adv_action,
                        const double *mid_next, const double *best_ask, const double *best_bid,
                        const double *buy_max, const double *sell_min,
                        double *reward, double *pnl_reward, double *inventory_reward,
                        double *fee_paid, uint8_t *fill_buy, uint8_t *fill_sell,
                        int64_t n, void *stream);

/* Batched TradingPolicy.forward (models/model.py:24-26): out[i] =
 * MLP(genomes[genome_idx[i]], states[i]).  Genome layout = parameters()
 * order W1[H,3] b1[H] W2[H,H] b2[H] W3[2,H] b3[2] (H*H+7H+2 floats).
 * genome_idx may be NULL (row i).  hidden in {8,16,32,64}. */
int sgmm_policy_forward(const float *genomes, int64_t genome_stride, int32_t hidden,
                        const int32_t *genome_idx, const float *states, float *out,
                        int64_t n, void *stream);

/* Batched AdversaryPolicy.forward (models/model.py:49-50): tanh outputs,
 * weights = the first 74 floats of each genome row (model.py:52-57). */
int sgmm_adversary_forward(const float *genomes, int64_t genome_stride,
                           const int32_t *genome_idx, const float *states, float *out,
                           int64_t n, void *stream);

/* Workspace bytes sgmm_rollout_fitness needs for this batch: n_inventory =
 * inv_max - inv_min + 1 inventory values, with_adversary != 0 when the batch
 * runs adversaries (adv_genomes / masters_adv non-NULL). (ABI 4) */
size_t sgmm_rollout_workspace_bytes(int32_t n_episodes, int64_t total_steps, int32_t n_inventory,
                                    int32_t with_adversary);
/* ABI 3 form: n_states = n_inventory, or 4 * n_inventory with the adversary
 * -- read as the adversary layout only when > 8, so an adversary batch with
 * fewer than 3 inventory values must be sized with sgmm_rollout_workspace_bytes. */
size_t sgmm_rollout_workspace_size(int32_t n_episodes, int64_t total_steps, int32_t n_states);

/* THE HOT PATH.  Fitness of every episode of the batch:
 * replaces Env/drl_engine.py:9-67 (evaluate_individual) as mapped by
 * Pool.starmap over the population (drl_engine.py:104-115).
 * fitness[e] = sum of step rewards (sequential float64 order), minus
 * idle_penalty if the episode never traded; trades[e] = steps with a fill.
 * adv_genomes may be NULL (no adversary, eps->adv ignored). */
int sgmm_rollout_fitness(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                         const sgmm_env_params *params,
                         const float *mm_genomes, int64_t mm_stride, int32_t hidden,
                         const float *adv_genomes, int64_t adv_stride,
                         double *fitness, int32_t *trades,
                         void *workspace, size_t workspace_bytes, void *stream);

/* Per-step trace of every episode (the recorder loop of
 * pipeline/agent_trainer.py:144-153 / main.py:63-90 / pipeline/evaluator.py:25-37,
 * batched).  Outputs are indexed by step_off[e] + t; any may be NULL.
 * off_a/off_b: MM action before the adversary; adv_a/adv_b: adversary deltas;
 * inventory/cash: after the step.  Also writes fitness/trades. */
int sgmm_rollout_trace(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                       const sgmm_env_params *params,
                       const float *mm_genomes, int64_t mm_stride, int32_t hidden,
                       const float *adv_genomes, int64_t adv_stride,
                       int32_t *off_a, int32_t *off_b, int32_t *adv_a, int32_t *adv_b,
                       int32_t *inventory, double *cash, double *reward, double *pnl_reward,
                       double *fee_paid, uint8_t *fill_buy, uint8_t *fill_sell,
                       float *raw_a, float *raw_b,
                       double *fitness, int32_t *trades, void *stream);

/* NeuroEvolution.ask (models/model.py:65-71) on device:
 * out[i,k] = master[k] + z(seed, stream_id, gen, i0+i, k) * (float)sigma,
 * z ~ N(0,1) from Philox4x32-10 + Box-Muller (counter-based, so any rank can
 * regenerate any individual).  sigma and gen are read ON DEVICE from `state`
 * (stream_id 0: sigma_mm, 1: sigma_adv; gen = state->gen), so a generation's
 * launches have fixed arguments and can be captured once in a HIP graph and
 * replayed.  out row stride out_stride. */
/* Device GA bookkeeping state (DRLEngine.train locals, drl_engine.py:84-89,
 * 143-160).  Initialise with sgmm_ga_state_init. */
typedef struct sgmm_ga_state {
    double  sigma_mm;      /* NeuroEvolution.sigma of the MM evolver */
    double  sigma_adv;     /* ... of the adversary evolver */
    double  best_val;      /* best_val_reward (-inf at start) */
    double  last_train_f;  /* best train fitness of the last generation */
    double  last_val_f;    /* validation reward of the last generation */
    int32_t no_improve;    /* no_improvement_gens */
    int32_t best_idx;      /* argmax of the last generation */
    int32_t adv_best_idx;  /* argmax of -fitness (adversary tell) */
    int32_t gen;           /* generations completed */
    int32_t improved;      /* last generation improved the validation reward */
    int32_t decayed;       /* last generation decayed sigma */
    int32_t patience;      /* 15 (drl_engine.py:155) */
    int32_t arrivals;      /* internal: workgroup arrival counter of a launch's generation tail (0 between launches) */
    double  decay;         /* 0.5 (drl_engine.py:156) */
} sgmm_ga_state;           /* 80 bytes */

/* History row written per generation (drl_engine.py:163-167). */
typedef struct sgmm_ga_history {
    double  train_f;
    double  val_f;
    double  sigma_after;
    int32_t train_trades;
    int32_t val_trades;
    int32_t best_idx;
    int32_t flags;         /* bit0 improved (checkpoint saved), bit1 sigma decayed */
} sgmm_ga_history;         /* 40 bytes */

int sgmm_ga_state_init(sgmm_ga_state *state, double sigma, int32_t patience, double decay,
                       void *stream);

int sgmm_ga_ask(const float *master, int64_t n_params, const sgmm_ga_state *state,
                uint32_t stream_id, uint64_t seed, int32_t i0, int32_t n,
                float *out, int64_t out_stride, void *stream);

/* NeuroEvolution.tell for both evolvers (model.py:73-76, drl_engine.py:119-125):
 * best = first index of max(fitness) (np.argmax; NaN counts as max),
 * adv_best = first index of max(-fitness).  The new master rows are written
 * into master_mm / master_adv either by copying row best of `pop_mm` /
 * `pop_adv` (host-supplied populations, may be NULL) or, when the pop
 * pointer is NULL, by regenerating the ask() of that index in place
 * (same seed/stream/gen as the ask).  P = global population size.
 * history: array of history_cap rows; row state->gen is written. */
int sgmm_ga_tell(sgmm_ga_state *state, const double *fitness, const int32_t *trades, int32_t P,
                 float *master_mm, const float *pop_mm, int64_t pop_mm_stride,
                 float *master_adv, const float *pop_adv, int64_t pop_adv_stride,
                 int64_t n_params_mm, int64_t n_params_adv, uint64_t seed,
                 sgmm_ga_history *history, int32_t history_cap, void *stream);

/* Validation bookkeeping after the best individual's validation rollout
 * (drl_engine.py:129-171): val_fitness/val_trades are read at index
 * state->best_idx when use_best_index (validation evaluated for the whole
 * population), else at 0.  On improvement master_mm is copied to best_master
 * (the checkpoint slot).  Applies sigma decay, completes history row
 * state->gen, then advances state->gen. */
int sgmm_ga_val_update(sgmm_ga_state *state, const double *val_fitness,
                       const int32_t *val_trades, int32_t use_best_index,
                       const float *master_mm, float *best_master, int64_t n_params_mm,
                       sgmm_ga_history *history, int32_t history_cap, void *stream);

/* One generation boundary in a single launch (single process or after the
 * fitness all-gather): tell (as sgmm_ga_tell, masters regenerated in place),
 * validation bookkeeping with the validation fitness of the whole population
 * (as sgmm_ga_val_update with use_best_index), then -- if next_pop_mm is not
 * NULL -- the ask() of the NEXT generation for individuals [i0, i0+n) with the
 * updated sigma (as sgmm_ga_ask; next_pop_adv likewise when master_adv).
 * Meant for modest P * n_params (one workgroup); use the separate entry points
 * for large populations.
 * Sharded inputs (multi-GPU, after an all-gather of per-rank records): with
 * shard_n > 0 the value of individual i in each of the four population arrays
 * is read at byte offset (i / shard_n) * shard_stride + (i % shard_n) *
 * sizeof(element) from its pointer; shard_n <= 0 means plain contiguous
 * arrays.  Every rank runs the same step on the gathered records, so masters
 * and sigma stay identical without a broadcast. */
int sgmm_ga_step(sgmm_ga_state *state, const double *fitness, const int32_t *trades,
                 const double *val_fitness, const int32_t *val_trades, int32_t P,
                 int32_t shard_n, int64_t shard_stride, float *master_mm, float *master_adv, float *best_master,
                 int64_t n_params_mm, int64_t n_params_adv, uint64_t seed,
                 sgmm_ga_history *history, int32_t history_cap,
                 float *next_pop_mm, float *next_pop_adv, int32_t i0, int32_t n, void *stream);

/* The current generation's ask() population, never materialized: episode e
 * evaluates individual i0 + genome[e] (adversary: i0 + adv[e], -1 = none)
 * whose genome is master + sigma * N(0,1) with the state's sigma and
 * generation -- exactly the rows sgmm_ga_ask would write -- generated inside
 * the rollout kernels (models/model.py:65-71 fused into drl_engine.py:104-115). */
typedef struct sgmm_asked_population {
    const sgmm_ga_state *state;
    const float *master_mm;   /* [genome_size(hidden)] */
    const float *master_adv;  /* [1250] or NULL (no adversary) */
    uint64_t seed;
    int32_t i0;               /* first individual of this rank's shard */
    int32_t pad_;
} sgmm_asked_population;     /* 40 bytes */

/* sgmm_rollout_fitness over the asked population (multi-rank shards: the
 * results then go through the all-gather and sgmm_ga_step). */
int sgmm_rollout_fitness_asked(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                               const sgmm_env_params *params, const sgmm_asked_population *pop,
                               int32_t hidden, double *fitness, int32_t *trades, void *workspace,
                               size_t workspace_bytes, void *stream);

/* One whole generation of DRLEngine.train on one process
 * (Env/drl_engine.py:92-171): the asked population's P training episodes
 * (eps 0..P-1, individual = genome[e]) and P validation episodes (eps
 * P..2P-1) in one rollout, and the generation boundary of sgmm_ga_step
 * (tell both evolvers, validation bookkeeping, sigma decay, history row
 * state->gen) run by the rollout's last workgroup.  fitness/trades: [2P].
 * Two kernel launches, no host synchronization; genome_size(hidden) <= 4096. */
int sgmm_generation(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                    const sgmm_env_params *params, sgmm_ga_state *state, float *master_mm,
                    float *master_adv, float *best_master, int32_t hidden, uint64_t seed,
                    int32_t P, double *fitness, int32_t *trades, sgmm_ga_history *history,
                    int32_t history_cap, void *workspace, size_t workspace_bytes, void *stream);

/* ------------------------------------------------------------------------
 * Several GA populations advanced together: one DRLEngine.train per
 * inventory penalty phi (the lambda sweep of pipeline/agent_trainer.py:136-137
 * called per phi at main.py:39-45; checkpoints/688981/agent_best_val_{phi}.pth)
 * or per asset (agent_trainer.py:168-173).  Population k keeps its own
 * master, sigma schedule, no-improvement counter, best validation reward,
 * history and Philox key -- exactly the state of an independent DRLEngine
 * run with seed seeds[k], so K populations in one launch reproduce K
 * separate runs bit for bit.  A HOST struct whose members point to device
 * memory; rows are contiguous per population.
 * ------------------------------------------------------------------------ */
typedef struct sgmm_populations {
    int32_t n_pop;              /* K */
    int32_t P;                  /* individuals per population (global, all ranks) */
    int32_t hidden;             /* TradingPolicy hidden width (every population) */
    int32_t history_cap;        /* history rows per population */
    sgmm_ga_state *states;      /* [K] (sgmm_ga_state_init each) */
    float *masters_mm;          /* [K][H*H+7H+2] */
    float *masters_adv;         /* [K][1250] or NULL (no adversary) */
    float *best_masters;        /* [K][H*H+7H+2] checkpoint slots (drl_engine.py:144-150) */
    const uint64_t *seeds;      /* [K] device: per-population Philox key */
    sgmm_ga_history *history;   /* [K][history_cap] */
    /* (ABI 5) optional, may be NULL: [K*P] device, the frontier kernel's walk
     * order of the TRAINING episodes for sgmm_generation_multi_best, read and
     * REWRITTEN on the device after each training launch (the walk-order
     * feedback; scheduling only, results do not depend on it).  The caller
     * seeds it with a permutation (e.g. a copy of train_eps->order), owns it
     * for the session and must not share it between concurrent calls.  NULL:
     * no feedback, train_eps->order is only read.  Every other entry point
     * ignores it.  The library never writes any sgmm_episodes array. */
    int32_t *walk_order;
} sgmm_populations;             /* 72 bytes */

/* One generation of K populations on one process.  Episodes: population k
 * owns episodes [2Pk, 2Pk+P) (training, individual genome[e]) and
 * [2Pk+P, 2P(k+1)) (validation, individual genome[e]); each episode's
 * params[param[e]] carries that population's phi / tick / fee.  The last
 * workgroup of each population runs its generation boundary (sgmm_ga_step).
 * fitness/trades: [K*2P], population-major.  Two kernel launches.
 * n_pop = 1 is sgmm_generation with seed = seeds[0]. */
int sgmm_generation_multi(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                          const sgmm_env_params *params, const sgmm_populations *pops,
                          double *fitness, int32_t *trades, void *workspace,
                          size_t workspace_bytes, void *stream);

/* A rank's shard of K asked populations (multi-GPU): population k owns
 * episodes [k*n_eps_pop, (k+1)*n_eps_pop) of the batch, individual
 * i0 + genome[e] of population k; fitness/trades [eps->n]. */
int sgmm_rollout_fitness_asked_multi(const sgmm_ticks *ticks, const sgmm_episodes *eps,
                                     const sgmm_env_params *params, const sgmm_populations *pops,
                                     int32_t i0, int32_t n_eps_pop, double *fitness,
                                     int32_t *trades, void *workspace, size_t workspace_bytes,
                                     void *stream);

/* One generation of K populations in the reference's order
 * (Env/drl_engine.py:92-171): the asked populations' training episodes
 * (train_eps: population k owns [kP, (k+1)P), individual genome[e]), the
 * tell of both evolvers in the training scan's tail (per population, its
 * last workgroup), then ONE validation episode per population on its new
 * master (sgmm_validate_multi) -- instead of validating every individual in
 * the training launch (sgmm_generation_multi).  Four kernel launches;
 * fitness/trades [K*P] (training), val_fitness/val_trades [K].  The workspace
 * must hold the larger of the two batches: sgmm_rollout_workspace_bytes(n,
 * steps, n_inventory, with_adversary) of each, with_adversary = masters_adv !=
 * NULL for the training batch and 0 for the validation batch.  With
 * pops->walk_order set, the training launch walks in that order and, when the
 * frontier kernel cuts some training episodes into halves (2.5-4 episodes per
 * SIMD) and the populations' episodes are of equal length, rewrites it on the
 * device after the launch so the next generation walks the lightest
 * populations whole (scheduling only: results do not depend on the order).
 * train_eps is read-only. */
int sgmm_generation_multi_best(const sgmm_ticks *ticks, const sgmm_episodes *train_eps,
                               const sgmm_episodes *val_eps, const sgmm_env_params *params,
                               const sgmm_populations *pops, double *fitness, int32_t *trades,
                               double *val_fitness, int32_t *val_trades, void *workspace,
                               size_t workspace_bytes, void *stream);

/* Validation of each population's current master (drl_engine.py:129-160),
 * after a tell (sgmm_ga_tell_multi, or the tail of sgmm_generation_multi_best):
 * val_eps holds one episode per population, episode k with genome[k] = k (row
 * k of masters_mm) and no adversary.  Then per population: improvement test
 * (strictly greater), checkpoint copy into best_masters, sigma decay, the
 * history row's validation fields, gen + 1.  Two kernel launches. */
int sgmm_validate_multi(const sgmm_ticks *ticks, const sgmm_episodes *val_eps,
                        const sgmm_env_params *params, const sgmm_populations *pops,
                        double *val_fitness, int32_t *val_trades, void *workspace,
                        size_t workspace_bytes, void *stream);

/* The tell of sgmm_ga_step_multi alone (NeuroEvolution.tell of both
 * evolvers, model.py:73-76, drl_engine.py:119-125): argmax, masters
 * regenerated, best index / training record into the state and history;
 * sgmm_validate_multi completes the generation (multi-GPU: every rank runs
 * both on the gathered training records). */
int sgmm_ga_tell_multi(const sgmm_populations *pops, const double *fitness, const int32_t *trades,
                       int64_t fit_pop_stride, int64_t trades_pop_stride, int32_t shard_n,
                       int64_t shard_stride, void *stream);

/* sgmm_ga_step for each of the K populations (one workgroup each, one
 * launch): population k reads its records at byte offset k * fit_pop_stride
 * from fitness / val_fitness and k * trades_pop_stride from trades /
 * val_trades, with the shard addressing of sgmm_ga_step (shard_n,
 * shard_stride) inside. */
int sgmm_ga_step_multi(const sgmm_populations *pops, const double *fitness, const int32_t *trades,
                       const double *val_fitness, const int32_t *val_trades,
                       int64_t fit_pop_stride, int64_t trades_pop_stride, int32_t shard_n,
                       int64_t shard_stride, void *stream);

/* Sequential float64 sum init + values[0] + values[1] + ... (device array,
 * result written to *out on the stream): the episode total of
 * Env/drl_engine.py:53 (total_reward += reward), evaluated in parallel and
 * bit-identical to the sequential loop.  The rollout uses the same routine. */
int sgmm_ordered_sum(const double *values, int64_t n, double init, double *out, void *stream);

/* ------------------------------------------------------------------------
 * Signal-bundle builder: raw snapshot / trade streams
 * of many trading days -> event bars -> SGU2 input windows -> per-step
 * bundle.  One workgroup per day.  Columns of day d occupy rows
 * [off[d], off[d+1]) and must be sorted by trade_time within the day (the
 * reference sorts with DataFrame.sort_values, HFTLoader.py:29-30).
 * ------------------------------------------------------------------------ */
typedef struct sgmm_day_streams {
    int32_t n_days;
    int32_t pad_;
    int64_t tick_total;        /* rows of the trade columns */
    const int64_t *snap_off;   /* [n_days + 1] */
    const int64_t *snap_time;  /* HHMMSSmmm */
    const double *bid, *ask, *bidvol, *askvol;  /* bidprice1 askprice1 bidvol1 askvol1 */
    const int64_t *tick_off;   /* [n_days + 1] */
    const int64_t *tick_time;
    const double *price, *volume;
    const int32_t *side;       /* +1 buy, -1 sell */
} sgmm_day_streams;            /* 104 bytes */

/* Event bars of every day, day d's events at rows snap_off[d] .. +n_events[d]
 * (capacity: the snapshot rows).  Columns as HFTMarketBase.event_df after the
 * as-of join (HFTLoader.py:26-63); statistics are NaN before the first trade. */
typedef struct sgmm_event_bars {
    int32_t *n_events;         /* [n_days] */
    int64_t *trade_time;
    double *ask, *bid, *p_buy_max, *p_sell_min, *v_buy_sum, *v_sell_sum, *vol_sum, *trade_count,
        *vwap_num;
} sgmm_event_bars;             /* 88 bytes */

size_t sgmm_event_bars_workspace_size(int64_t total_ticks);

/* HFTMarketBase (loaders/HFTLoader.py:26-63) for every day. */
int sgmm_event_bars_build(const sgmm_day_streams *in, const sgmm_event_bars *out, void *workspace,
                          size_t workspace_bytes, void *stream);

/* SGU2DataPro.gen_dataset(event_step=19, time_steps=10) (HFTLoader.py:139-169)
 * for every day: windows of day d at rows win_off[d] .. +n_windows[d] of
 * X[., 10] / y (float32).  At most 4096 bars (19-event groups) per day. */
int sgmm_bar_windows(const sgmm_event_bars *ev, int32_t n_days, const int64_t *snap_off,
                     const int64_t *win_off, float *X, float *y, int32_t *n_windows,
                     int64_t max_bars_per_day, void *stream);

/* load_signals_bundle's step loop (pipeline/agent_trainer.py:45-78): day d
 * uses its last n_samples[d] sampled events (every 19th) and writes
 * n_samples[d]-1 steps at step_off[d]: mid at the next sample, ask/bid at the
 * sample, buy_max/sell_min over the inclusive .loc window between samples. */
int sgmm_step_bundle(const sgmm_event_bars *ev, int32_t n_days, const int64_t *snap_off,
                     const int32_t *n_samples, const int64_t *step_off, int32_t max_steps,
                     double *mid, double *ask, double *bid, double *buy_max, double *sell_min,
                     void *stream);

/* ------------------------------------------------------------------------
 * SGU2 inference
 * ------------------------------------------------------------------------ */

/* SGU2.predict (models/GateUnits.py:116-120): SGU2Model.forward in eval mode
 * (GateUnits.py:42-54 -- nn.LSTM(1, hidden) over each window, last hidden
 * state, Linear(hidden, 1)) for n windows X[n, time_steps, 1] (float32, the
 * windows of sgmm_bar_windows).  weights: float32 in state_dict order --
 * lstm.weight_ih_l0[4H,1], lstm.weight_hh_l0[4H,H], lstm.bias_ih_l0[4H],
 * lstm.bias_hh_l0[4H], fc.weight[1,H], fc.bias[1].  mean/std: the float32
 * StandardScaler3D fit (utils/scaler.py:9-18; agent_trainer.py:43 scales
 * before predict), applied in the kernel, or both NULL for unscaled input.
 * out: float32[n].  hidden in {10, 16, 32}. */
int sgmm_sgu2_forward(const float *weights, int32_t hidden, const float *X, int64_t n,
                      int32_t time_steps, const float *mean, const float *std, float *out,
                      void *stream);

/* ------------------------------------------------------------------------
 * Launch-plan overrides (ABI 5), for tests and A/B experiments.  The shipped
 * library reads no environment variable; its launch plan (policy kernel,
 * chunk groups, lane split, scan width, spill budget) follows the measured
 * rules documented in DESIGN.md unless overridden here.  Overrides are
 * process-wide and apply to launches ENQUEUED after the call (a captured HIP
 * graph keeps the plan it was captured with); set them before building
 * workspaces, since the workspace size follows the plan.  value < 0 restores
 * the default rule.  sgmm_plan_set returns 0 or SGMM_ERR_ARG (unknown knob);
 * sgmm_plan_get returns the override, -1 for the default rule, or INT32_MIN for
 * an unknown knob.  (A build with -DSGMM_EXPERIMENTS also takes the initial
 * values from the SGMM_* environment variables named in DESIGN.md.)
 * ------------------------------------------------------------------------ */
enum {
    SGMM_PLAN_POLICY_PATH = 0,   /* 0 auto, 1 frontier, 2 MFMA table, 3 VALU table */
    SGMM_PLAN_GROUPS = 1,        /* frontier chunk groups per episode, 1..16 */
    SGMM_PLAN_LANE_SPLIT = 2,    /* frontier waves per walk: 1, 2 or 4 */
    SGMM_PLAN_TAIL = 3,          /* 0: no split tail walks (every walk whole) */
    SGMM_PLAN_FOUR = 4,          /* 0: no four-walk rule */
    SGMM_PLAN_MIN_EPS = 5,       /* frontier kernel from this many episodes */
    SGMM_PLAN_TABLE_SP = 6,      /* 0 / 1: state-parallel table off / forced */
    SGMM_PLAN_SCAN_THREADS = 7,  /* path-scan workgroup: 64, 256, 512 or 1024 */
    SGMM_PLAN_REORDER_WEIGHTS = 8, /* walk-order scores: whole << 8 | split */
    SGMM_PLAN_SPILL = 9,         /* frontier spill deadline, us after a walk's start (0: off) */
    SGMM_PLAN_SEQ_SUM = 10,      /* path-scan episode sums: 0 exact parallel method, 1 sequential chain */
    SGMM_PLAN_FUSED_SCAN = 11,   /* frontier launches: 0 separate path scan, 1 scans fused into the walks */
    SGMM_PLAN_LANES_SCAN = 12,   /* frontier path scan: 1 = 2-4 episodes per workgroup, chains in lanes (2 / 4 force
                                    the count); 0 = one episode per wave */
    SGMM_PLAN_N = 13
};
int sgmm_plan_set(int32_t knob, int32_t value);
int sgmm_plan_get(int32_t knob);

/* Kernel timing for benchmarks / diagnostics (not on by default).
 * While enabled, every kernel the library launches is bracketed by a pair of
 * hipEvents recorded on its stream.  sgmm_profile_read waits for the recorded
 * events, writes up to max_kinds entries (name[i] = names + 48*i,
 * NUL-terminated; total_ms[i]; count[i]) and clears the record.  Returns the
 * number of kernel kinds written, or < 0 on error. */
int sgmm_profile_enable(int enable);
int sgmm_profile_read(int max_kinds, char *names, double *total_ms, int64_t *count);

#ifdef __cplusplus
}
#endif

#endif /* SGMM_H */
