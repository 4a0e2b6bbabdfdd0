/*
 * flsim_oracle.c -- CPU restatement of the reference's integer / fp32-elementwise hot-path
 * algorithms.  TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker.  The product path
 * (fl-distributed-delay_amd/) never links or calls it.
 *
 * Pinned against golden vectors produced by the reference itself (tests/golden/make_golden.py
 * runs /root/reference/main.py's loop + FL/agents.py in this container).
 *
 * Restated algorithms (reference file:line):
 *   oracle_schedule_run   main.py:119-123 (state), 126,137 (loops), 150-166 (slow worker +
 *                         pesky_worker_grads FIFO), 167-178 (fast + throttle), 180-181 (decrement)
 *   oracle_cascade_mean   main.py:23-25 rule(): torch.stack(entries).mean(0) on CPU; torch 2.10
 *                         ATen SumKernel multi_row_sum cascade (4 levels), then / k
 *   oracle_adam_step      agents.py:9-21 Central.update_model -> torch.optim.Adam (main.py:106),
 *                         torch 2.10 _single_tensor_adam CPU op order
 *   oracle_philox / oracle_dropout_keep / oracle_sample_slots
 *                         the build's counter-based replacement for the reference's RNG draws
 *                         (main.py:85-88 RandomSampler, models.py:17,23 nn.Dropout); spec in DESIGN.md
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off: every fma below is explicit).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al. 2011), counter = (c0,c1,c2,c3), key = (k0,k1).                 */
/* ------------------------------------------------------------------------------------------ */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0;
        uint32_t n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

/* word `e & 3` of philox(ctr = (e>>2, t, worker, site), key = (seed_lo, seed_hi)) */
uint32_t oracle_philox(uint64_t seed, uint32_t t, uint32_t worker, uint32_t site, uint32_t e) {
    uint32_t c[4] = { e >> 2, t, worker, site };
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return c[e & 3];
}

/* keep mask for `count` consecutive elements starting at element e0 (NCHW order within the
 * worker's batch); keep iff u32 >= threshold.  threshold = p * 2^32.                          */
void oracle_dropout_keep(uint64_t seed, uint32_t t, uint32_t worker, uint32_t site,
                         uint32_t threshold, uint64_t e0, uint64_t count, uint8_t* keep) {
    uint64_t e = e0;
    uint64_t end = e0 + count;
    while (e < end) {
        uint32_t c[4] = { (uint32_t)(e >> 2), t, worker, site };
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (uint32_t w = (uint32_t)(e & 3); w < 4 && e < end; ++w, ++e)
            keep[e - e0] = c[w] >= threshold ? 1 : 0;
    }
}

/* sample slots j = 0..n-1 of worker-step (t, worker): u32 % len */
void oracle_sample_slots(uint64_t seed, uint32_t t, uint32_t worker, uint32_t site,
                         uint32_t len, uint32_t n, uint32_t* out) {
    for (uint32_t j = 0; j < n; ++j)
        out[j] = oracle_philox(seed, t, worker, site, j) % len;
}

/* ------------------------------------------------------------------------------------------ */
/* Schedule scan: main.py:119-181 restated.  Slow workers = those with delay[i] > 0; the       */
/* reference has exactly one (i = n-1, delay = --delay).  Each slow worker owns a FIFO.         */
/*   per epoch outputs:                                                                        */
/*     computes[t*n + i]   1 if worker i ran fwd_bkwd in epoch t                                */
/*     appended[t*n + i]   1 if worker i's entry went into weight_ups (fast: = computes;         */
/*                         slow: popped a stale entry)                                         */
/*     stale_src[t*n + i]  epoch whose gradient the popped entry holds (-1 if none)            */
/*     c_t[t]              fast workers that computed (== losses appended, main.py:172)        */
/*     s_t[t]              stale entries appended                                               */
/*     window_end[t], gone_end[t]   throttle state after the epoch                             */
/*   returns 0, or 1 when main.py would raise (d == 0 at t>0: ZeroDivisionError; empty           */
/*   weight_ups: IndexError in rule()), with *fail_epoch set.                                  */
/* ------------------------------------------------------------------------------------------ */
int oracle_schedule_run(int32_t n, const int32_t* delay, int32_t throttle, int32_t max_throttle,
                        int64_t n_epochs, uint8_t* computes, uint8_t* appended, int64_t* stale_src,
                        int32_t* c_t, int32_t* s_t, int32_t* window_end, uint8_t* gone_end,
                        int64_t* fail_epoch) {
    int64_t throttle_window = 0;              /* main.py:121 */
    int slow_guy_gone = 0;                    /* main.py:123 */
    /* FIFO per slow worker: pushed epochs; never more than 2 deep for constant delay */
    int64_t* fifo = (int64_t*)calloc((size_t)n * 4, sizeof(int64_t));
    int32_t* fifo_len = (int32_t*)calloc((size_t)n, sizeof(int32_t));
    int rc = 0;
    for (int64_t t = 0; t < n_epochs; ++t) {
        int32_t c = 0, s = 0;
        for (int32_t i = 0; i < n; ++i) {
            int64_t idx = t * n + i;
            computes[idx] = 0; appended[idx] = 0; stale_src[idx] = -1;
            if (delay[i] != 0) {                              /* main.py:150 */
                slow_guy_gone = 0;                            /* main.py:151 */
                int64_t popped = -1;
                const int64_t d = delay[i] < 0 ? -(int64_t)delay[i] : (int64_t)delay[i];
                if (t == 0) {                                 /* main.py:153-157 */
                    computes[idx] = 1;
                    fifo[i * 4 + fifo_len[i]++] = t;
                } else if (t % d == 0) {                      /* main.py:158-162 */
                    computes[idx] = 1;
                    fifo[i * 4 + fifo_len[i]++] = t;
                    popped = fifo[i * 4];
                    for (int q = 1; q < fifo_len[i]; ++q) fifo[i * 4 + q - 1] = fifo[i * 4 + q];
                    fifo_len[i]--;
                }
                if (popped >= 0) {                            /* main.py:164-166 */
                    appended[idx] = 1; stale_src[idx] = popped; s++;
                    slow_guy_gone = 1;
                }
            } else {
                if (throttle_window <= 0) {                   /* main.py:168-172 */
                    computes[idx] = 1; appended[idx] = 1; c++;
                    if (throttle) {                           /* main.py:174-178 */
                        throttle_window = 1;
                        if (!slow_guy_gone) {
                            throttle_window *= 2;
                            if (throttle_window > max_throttle) throttle_window = max_throttle;
                        }
                    }
                }
            }
            if (throttle_window > 0) throttle_window -= 1;   /* main.py:180-181 */
        }
        c_t[t] = c; s_t[t] = s;
        window_end[t] = (int32_t)throttle_window; gone_end[t] = (uint8_t)slow_guy_gone;
        if (c + s == 0) { rc = 1; if (fail_epoch) *fail_epoch = t; break; }   /* rule(): IndexError */
    }
    free(fifo); free(fifo_len);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Cascade mean, torch 2.10 CPU: sum over the stacked dim with ATen's multi_row_sum           */
/* (num_levels = 4, level_power = max(4, ceil_log2(k) / 4)), accumulated in fp32, then / k.    */
/* entries: k pointers to P floats.                                                            */
/* ------------------------------------------------------------------------------------------ */
static int64_t ceil_log2_i64(uint64_t x) {
    if (x <= 1) return 0;
    int64_t r = 0; uint64_t v = x - 1;
    while (v) { r++; v >>= 1; }
    return r;
}

/* multi_row_sum over `size` rows for one column; row r's value is entries[first + r*stride][e] */
static float multi_row_sum_col(const float* const* entries, int64_t first, int64_t stride,
                               int64_t size, int64_t e) {
    const int64_t num_levels = 4;
    int64_t level_power = ceil_log2_i64((uint64_t)size) / num_levels;
    if (level_power < 4) level_power = 4;
    const int64_t level_step = (int64_t)1 << level_power;
    const int64_t level_mask = level_step - 1;
    float acc[4] = { 0.f, 0.f, 0.f, 0.f };
    int64_t i = 0;
    for (; i + level_step <= size;) {
        for (int64_t j = 0; j < level_step; ++j, ++i) acc[0] += entries[first + i * stride][e];
        for (int64_t j = 1; j < num_levels; ++j) {
            acc[j] += acc[j - 1];
            acc[j - 1] = 0.f;
            const int64_t mask = level_mask << (j * level_power);
            if ((i & mask) != 0) break;
        }
    }
    for (; i < size; ++i) acc[0] += entries[first + i * stride][e];
    for (int64_t j = 1; j < num_levels; ++j) acc[0] += acc[j];
    return acc[0];
}

/* row_sum: the k rows viewed as (k/4, 4) -> four interleaved multi_row_sum streams, leftovers
 * into stream 0, then s0 + s1 + s2 + s3.                                                      */
static float row_sum_col(const float* const* entries, int64_t k, int64_t e) {
    const int64_t sz = k / 4;
    float ps[4];
    for (int q = 0; q < 4; ++q) ps[q] = multi_row_sum_col(entries, q, 4, sz, e);
    for (int64_t i = sz * 4; i < k; ++i) ps[0] += entries[i][e];
    for (int q = 1; q < 4; ++q) ps[0] += ps[q];
    return ps[0];
}

/* One parameter tensor of P elements: torch's vectorized_outer_sum runs multi_row_sum on whole
 * 32-column blocks and row_sum on the remaining P % 32 columns (measured on torch 2.10 CPU; the
 * parallel split over columns rounds chunk edges to 128 bytes, so only the global tail differs). */
void oracle_cascade_mean(const float* const* entries, int64_t k, int64_t P, float* out) {
    const float kf = (float)k;
    const int64_t tail0 = (P / 32) * 32;
    for (int64_t e = 0; e < P; ++e) {
        float s = e < tail0 ? multi_row_sum_col(entries, 0, 1, k, e) : row_sum_col(entries, k, e);
        out[e] = s / kf;
    }
}

/* Convenience for the reference's weight_ups shape: c copies of S followed by n_stale stale
 * entries (each its own array).  Same arithmetic as oracle_cascade_mean.                      */
void oracle_cascade_mean_rep(const float* S, int64_t c, const float* const* stale, int64_t n_stale,
                             int64_t P, float* out) {
    int64_t k = c + n_stale;
    const float** ent = (const float**)malloc(sizeof(float*) * (size_t)k);
    for (int64_t i = 0; i < c; ++i) ent[i] = S;
    for (int64_t i = 0; i < n_stale; ++i) ent[c + i] = stale[i];
    oracle_cascade_mean(ent, k, P, out);
    free(ent);
}

/* ------------------------------------------------------------------------------------------ */
/* Adam, torch 2.10 _single_tensor_adam on CPU (foreach=None -> single tensor for CPU params). */
/*   exp_avg.lerp_(grad, 1-beta1)          : m = fma(w, g - m, m)       (w = (float)(1-beta1)) */
/*   exp_avg_sq.mul_(beta2)                : v = v * (float)beta2                             */
/*   .addcmul_(grad, grad, value=1-beta2)  : v = fma((float)(1-beta2) * g, g, v)               */
/*   denom = (sqrt(v) / (float)sqrt(bc2)).add_(eps)                                             */
/*   param.addcdiv_(m, denom, value=-step_size) : p = p + ((float)(-step_size) * m) / denom    */
/* step is the count AFTER increment; bias corrections in double like the Python code.         */
/* The sqrt here is correctly rounded; torch's vectorised CPU sqrt is not always (1 ulp).      */
/* ------------------------------------------------------------------------------------------ */
void oracle_adam_step(float* p, float* m, float* v, const float* g, int64_t P, int64_t step,
                      double lr, double beta1, double beta2, double eps) {
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const double step_size = lr / bc1;
    const float w1 = (float)(1.0 - beta1);
    const float b2 = (float)beta2;
    const float w2 = (float)(1.0 - beta2);
    const float bc2s = (float)sqrt(bc2);
    const float epsf = (float)eps;
    const float neg_ss = (float)(-step_size);
    for (int64_t e = 0; e < P; ++e) {
        const float gi = g[e];
        float mi = fmaf(w1, gi - m[e], m[e]);
        float vi = v[e] * b2;
        vi = fmaf(w2 * gi, gi, vi);
        float den = sqrtf(vi) / bc2s + epsf;
        p[e] = p[e] + (neg_ss * mi) / den;
        m[e] = mi; v[e] = vi;
    }
}
