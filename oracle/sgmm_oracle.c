/*
 * sgmm_oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library, the
 * host package) links, loads or calls this file.  It is used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only as the
 * checker / the timed CPU baseline -- never as the thing measured or shipped.
 *
 * Parity: pinned against golden vectors generated from the imported
 * reference (tests/golden/gen_golden.py) -- see DESIGN.md "Oracle".
 *
 * What it restates (reference paths relative to the reference repo root):
 *   orc_env_step          Env/market_env.py:22-67   FTPEnv.step
 *   orc_policy_forward    models/model.py:5-36      TradingPolicy.forward
 *   orc_adversary_forward models/model.py:38-57     AdversaryPolicy.forward
 *   orc_evaluate          Env/drl_engine.py:9-67    evaluate_individual
 *
 * Numerics contract (shared with the HIP kernels):
 *   - prices / cash / reward: float64, evaluated with the reference's operation
 *     order and NO fused multiply-add (build with -ffp-contract=off);
 *   - MLP: float32, every dot product is the k-ordered fused chain
 *       acc = bias; acc = fmaf(w[k], x[k], acc) for k = 0..K-1
 *     (torch's MKL order is unspecified; rounded actions are pinned by the
 *     golden fixtures, raw outputs agree to a few ulp);
 *   - actions: rintf(raw * scale) (round half to even, as np.round).
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <limits.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* Episode parameters.  Layout mirrors include/sgmm.h's sgmm_env_params. */
typedef struct {
    double  phi;          /* inventory penalty (market_env.py:10) */
    double  tick;         /* tick size (market_env.py:11) */
    double  fee;          /* fee rate (market_env.py:9) */
    double  idle_penalty; /* subtracted when an episode never trades (drl_engine.py:64-65) */
    int32_t i_max;        /* market_env.py:14 */
    int32_t i_min;        /* market_env.py:15 */
    float   act_scale;    /* drl_engine.py:39 (5.0) */
    float   adv_scale;    /* drl_engine.py:48 (1.0) */
} orc_params;

/* Optional per-step trace; any pointer may be NULL. */
typedef struct {
    int32_t *off_a, *off_b;       /* MM action after rounding (before adversary) */
    int32_t *adv_a, *adv_b;       /* adversary deltas (0 without adversary) */
    int32_t *inventory;           /* inventory after the step */
    double  *cash;                /* cash after the step */
    double  *reward, *pnl, *fee_paid;
    uint8_t *fill_buy, *fill_sell;
    float   *raw_a, *raw_b;       /* raw MLP outputs */
} orc_trace;

/* float -> int conversion used for actions: saturating, NaN -> INT32_MIN
 * (x86 cvtt semantics, which is what numpy's astype(int) yields for NaN). */
static int32_t act_to_int(float r)
{
    if (r != r) return INT32_MIN;
    if (r >= 2147483520.0f) return INT32_MAX;
    if (r <= -2147483648.0f) return INT32_MIN;
    return (int32_t)r;
}

/* ReLU on the bit pattern, max(bits, 0) as int32.  The kernels use
 * v_med3_f32(a, 0, +inf) instead (sgmm_device.h relu); the two agree for every
 * non-NaN input except the sign of a zero (-0.0 -> +0.0 here, -0.0 or +0.0
 * there), which changes no dot product's value beyond the sign of an exact
 * zero and so no action.  Both equal torch's relu on non-NaN inputs; NaN
 * pre-activations (only NaN state inputs produce them) are outside the
 * parity domain, where the two forms may differ. */
static float relu32(float a)
{
    int32_t b;
    memcpy(&b, &a, sizeof b);
    b = b > 0 ? b : 0;
    memcpy(&a, &b, sizeof a);
    return a;
}

/* ---- FTPEnv.step (Env/market_env.py:22-67) -------------------------------- */
/* out4 = {reward, pnl_reward, inventory_reward, fee_paid}; fills = {buy, sell} */
int orc_env_step(const orc_params *p, int32_t *inv, double *cash,
                 int32_t off_a, int32_t off_b, int has_adv, int32_t adv_a, int32_t adv_b,
                 double mid_next, double best_ask, double best_bid,
                 double buy_max, double sell_min, double *out4, int32_t *fills)
{
    if (has_adv) { off_a += adv_a; off_b += adv_b; }          /* market_env.py:25-28 */
    const double quote_ask = best_ask + (double)off_a * p->tick;  /* :30 */
    const double quote_bid = best_bid - (double)off_b * p->tick;  /* :31 */
    const int32_t pos = *inv;
    const int buy = (pos < p->i_max) && (quote_bid >= sell_min);   /* :34,37 */
    const int sell = (pos > p->i_min) && (quote_ask <= buy_max);   /* :35,38 */
    double pnl = 0.0, fees = 0.0, c = *cash;
    int32_t q = pos;
    if (buy) {                                                     /* :44-49 */
        const double f = quote_bid * p->fee;
        q += 1;
        c -= (quote_bid + f);
        pnl += (mid_next - quote_bid) - f;
        fees += f;
    }
    if (sell) {                                                    /* :50-55 */
        const double f = quote_ask * p->fee;
        q -= 1;
        c += (quote_ask - f);
        pnl += (quote_ask - mid_next) - f;
        fees += f;
    }
    const double pen = p->phi * (double)(q < 0 ? -q : q);         /* :57 */
    *inv = q;
    *cash = c;
    out4[0] = pnl - pen;                                           /* :58 */
    out4[1] = pnl;
    out4[2] = -pen;
    out4[3] = fees;
    fills[0] = buy;
    fills[1] = sell;
    return 0;
}

/* ---- TradingPolicy forward (models/model.py:5-36), canonical order -------- */
/* genome layout = parameters() order: W1[H,3] b1[H] W2[H,H] b2[H] W3[2,H] b3[2] */
void orc_policy_forward(const float *g, int H, const float *x, float *out)
{
    const float *W1 = g, *b1 = W1 + 3 * H, *W2 = b1 + H, *b2 = W2 + H * H;
    const float *W3 = b2 + H, *b3 = W3 + 2 * H;
    float h1[256], h2[256];
    for (int j = 0; j < H; ++j) {
        float a = b1[j];
        a = fmaf(W1[3 * j + 0], x[0], a);
        a = fmaf(W1[3 * j + 1], x[1], a);
        a = fmaf(W1[3 * j + 2], x[2], a);
        h1[j] = relu32(a);
    }
    for (int j = 0; j < H; ++j) {
        float a = b2[j];
        for (int k = 0; k < H; ++k) a = fmaf(W2[j * H + k], h1[k], a);
        h2[j] = relu32(a);
    }
    for (int o = 0; o < 2; ++o) {
        float a = b3[o];
        for (int j = 0; j < H; ++j) a = fmaf(W3[o * H + j], h2[j], a);
        out[o] = a;
    }
}

/* ---- AdversaryPolicy forward (models/model.py:38-57) ---------------------- */
/* Uses the first 74 floats of the genome (fc.0.weight[12,3], fc.0.bias[12],
 * fc.2.weight[2,12], fc.2.bias[2]) -- the reference's set_weights copies the
 * leading 74 floats of a TradingPolicy-layout genome (model.py:49-54,63). */
void orc_adversary_forward(const float *g, const float *x, float *out)
{
    const float *W1 = g, *b1 = g + 36, *W2 = g + 48, *b2 = g + 72;
    float h[12];
    for (int j = 0; j < 12; ++j) {
        float a = b1[j];
        a = fmaf(W1[3 * j + 0], x[0], a);
        a = fmaf(W1[3 * j + 1], x[1], a);
        a = fmaf(W1[3 * j + 2], x[2], a);
        h[j] = relu32(a);
    }
    for (int o = 0; o < 2; ++o) {
        float a = b2[o];
        for (int j = 0; j < 12; ++j) a = fmaf(W2[o * 12 + j], h[j], a);
        out[o] = tanhf(a);
    }
}

/* ---- evaluate_individual (Env/drl_engine.py:9-67) ------------------------- */
/* s1n/s2n: the normalised signals (drl_engine.py:33-34), already float32. */
double orc_evaluate(const float *mm, int H, const float *adv,
                    const float *s1n, const float *s2n,
                    const double *mid_next, const double *best_ask, const double *best_bid,
                    const double *buy_max, const double *sell_min, int64_t T,
                    const orc_params *p, int32_t *trades_out, const orc_trace *tr)
{
    int32_t inv = 0, trades = 0;
    double cash = 0.0, total = 0.0;
    float flag_buy = 0.0f, flag_sell = 0.0f;
    for (int64_t t = 0; t < T; ++t) {
        const float x[3] = { s1n[t], s2n[t], (float)((double)inv / 2.0) };  /* :33-35 */
        float raw[2];
        orc_policy_forward(mm, H, x, raw);
        const int32_t oa = act_to_int(rintf(raw[0] * p->act_scale));      /* :38-39 */
        const int32_t ob = act_to_int(rintf(raw[1] * p->act_scale));
        int32_t da = 0, db = 0;
        if (adv) {                                                          /* :43-48 */
            const float xa[3] = { (float)((double)inv / 2.0), flag_sell, flag_buy };
            float ar[2];
            orc_adversary_forward(adv, xa, ar);
            da = act_to_int(rintf(ar[0] * p->adv_scale));
            db = act_to_int(rintf(ar[1] * p->adv_scale));
        }
        double o4[4];
        int32_t fills[2];
        orc_env_step(p, &inv, &cash, oa, ob, adv != NULL, da, db,
                     mid_next[t], best_ask[t], best_bid[t], buy_max[t], sell_min[t], o4, fills);
        total += o4[0];                                                     /* :54 */
        flag_buy = fills[0] ? 1.0f : 0.0f;                                  /* :57-58 */
        flag_sell = fills[1] ? 1.0f : 0.0f;
        if (fills[0] || fills[1]) trades += 1;                              /* :60-61 */
        if (tr) {
            if (tr->off_a) tr->off_a[t] = oa;
            if (tr->off_b) tr->off_b[t] = ob;
            if (tr->adv_a) tr->adv_a[t] = da;
            if (tr->adv_b) tr->adv_b[t] = db;
            if (tr->inventory) tr->inventory[t] = inv;
            if (tr->cash) tr->cash[t] = cash;
            if (tr->reward) tr->reward[t] = o4[0];
            if (tr->pnl) tr->pnl[t] = o4[1];
            if (tr->fee_paid) tr->fee_paid[t] = o4[3];
            if (tr->fill_buy) tr->fill_buy[t] = (uint8_t)fills[0];
            if (tr->fill_sell) tr->fill_sell[t] = (uint8_t)fills[1];
            if (tr->raw_a) tr->raw_a[t] = raw[0];
            if (tr->raw_b) tr->raw_b[t] = raw[1];
        }
    }
    if (trades == 0) total -= p->idle_penalty;                              /* :64-65 */
    if (trades_out) *trades_out = trades;
    return total;
}

/* Batch of episodes (the population loop of drl_engine.py:104-115).
 * Episode e uses genome ep_genome[e] (row of mm, stride G), adversary
 * ep_adv[e] (row of adv with stride Ga, or -1), ticks [ep_off[e], +ep_len[e])
 * and params[ep_param[e]].  n_threads > 1 uses OpenMP when built with it. */
void orc_evaluate_batch(const float *mm, int H, int64_t G,
                        const float *adv, int64_t Ga,
                        const float *s1n, const float *s2n,
                        const double *mid_next, const double *best_ask, const double *best_bid,
                        const double *buy_max, const double *sell_min,
                        int32_t n_ep, const int32_t *ep_genome, const int32_t *ep_adv,
                        const int64_t *ep_off, const int64_t *ep_len, const int32_t *ep_param,
                        const orc_params *params, double *fitness, int32_t *trades, int n_threads)
{
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1) if (n_threads > 1)
#endif
    for (int32_t e = 0; e < n_ep; ++e) {
        const int64_t o = ep_off[e];
        const float *a = (adv && ep_adv && ep_adv[e] >= 0) ? adv + (int64_t)ep_adv[e] * Ga : NULL;
        fitness[e] = orc_evaluate(mm + (int64_t)ep_genome[e] * G, H, a, s1n + o, s2n + o,
                                  mid_next + o, best_ask + o, best_bid + o, buy_max + o, sell_min + o,
                                  ep_len[e], &params[ep_param[e]], &trades[e], NULL);
    }
    (void)n_threads;
}

int orc_abi_version(void) { return 1; }
