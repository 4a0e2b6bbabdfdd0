// rule()'s summation order as a tiny program (reference: main.py:23-25, torch.stack(weight_ups)
// .mean(0) on CPU = ATen's cascade sum over the stacked dim, then / k).
//
// The k entries of weight_ups are either x (the aliased S_t of every fast worker, main.py:172) or a
// stale FIFO entry y_q (main.py:161-165; q = which distinct array).  The cascade order is fixed by
// k and by WHERE the y entries sit, not by the values, so the host turns (k, event positions) into
// a straight-line program once per server step and every element runs the same program with its
// own x and y values: all control flow is uniform (scalar), only the adds are per element.
//
// ATen multi_row_sum (torch 2.10, restated in oracle/flsim_oracle.c multi_row_sum_col): four
// accumulators, level step L = 2^lp, lp = max(4, ceil_log2(rows) / 4); rows go into a0; after each
// full block of L rows a1 += a0, a0 = 0; when the row count is a multiple of L^2 also a2 += a1,
// a1 = 0; of L^3 also a3 += a2, a2 = 0; rows past the last full block stay in a0; result
// ((a0 + a1) + a2) + a3.  The last numel % 32 elements of every tensor use row_sum instead: the k
// rows viewed as (k/4, 4), stream q = rows 4r + q by multi_row_sum, leftover rows added to stream
// 0, then ((s0 + s1) + s2) + s3.
//
// Runs of x-only structure are compressed exactly:
//   a pure block (L x's, a0 = 0 at its start) leaves a0 = bx = seq_sum(x, L): it is "a1 += bx";
//   a pure level-1 group (L pure blocks, a1 = 0 at its start) is "a2 += g1", g1 = seq_sum(bx, L);
//   a pure level-2 group is "a3 += g2", g2 = seq_sum(g1, L);
// where seq_sum(v, n) = ((0 + v) + v) ... (n adds from +0), the same roundings the cascade does.
#pragma once
#include <stdint.h>

namespace flsim {

enum CascOp : int32_t {
    COP_END = 0,   // result = r0
    COP_X = 1,     // a0 += x, n times
    COP_Y = 2,     // a0 += y[n]
    COP_C1 = 3,    // a1 += a0, a0 = 0
    COP_C2 = 4,    // a2 += a1, a1 = 0
    COP_C3 = 5,    // a3 += a2, a2 = 0
    COP_BX = 6,    // a1 += bx, n times (n pure blocks, no level-1 boundary inside)
    COP_G1 = 7,    // a2 += g1, n times (n pure level-1 groups, no level-2 boundary inside)
    COP_G2 = 8,    // a3 += g2, n times
    COP_FIN = 9,   // r[n] = ((a0 + a1) + a2) + a3; a* = 0
    COP_LX = 10,   // r0 += x           (row_sum leftover rows)
    COP_LY = 11,   // r0 += y[n]
    COP_RS = 12,   // r0 = ((r0 + r1) + r2) + r3
    // fused pairs (emitted by the builder's peephole; halve the ops of event blocks)
    COP_XY = 13,   // a0 += x, n times; a0 += y[q]       (n = bits 4..15, q = bits 16..31)
    COP_XC1 = 14,  // a0 += x, n times; a1 += a0, a0 = 0
    COP_BXC2 = 15, // a1 += bx, n times; a2 += a1, a1 = 0
};
constexpr int COP_SHIFT = 4;
constexpr int CASC_PAD = 8;             // words the interpreter may fetch past a COP_END
constexpr int CASC_MAX_K = 1 << 19;     // lp == 4 for the whole sequence and its row_sum streams

// program header (info[]) written by build_cascade_program
struct CascInfo {
    int32_t len;        // words
    int32_t tail_off;   // start of the row_sum program (tensor tails)
    int32_t need;       // bit 0: bx, bit 1: g1, bit 2: g2
    int32_t lp;         // level power (4)
};

// ---- host: program builder --------------------------------------------------------------------
// Events: entry positions pos[j] (strictly increasing) holding array arr[j]; every other position
// is x.  Returns the program length, or -1 (bad events), -2 (capacity), -3 (k out of range).
struct CascEmitter {
    int32_t* out;
    int cap, len = 0, need = 0;
    bool ok = true;
    int stream_start = 0;     // no fusion across a program boundary
    void put(int op, int n = 0) {
        if (op == COP_BX) need |= 1;
        if (op == COP_G1) need |= 3;
        if (op == COP_G2) need |= 7;
        if (len > stream_start) {         // peephole: fuse with the previous word
            const uint32_t prev = (uint32_t)out[len - 1];
            const int pop = (int)(prev & 15u), pn = (int)(prev >> COP_SHIFT);
            if (op == COP_Y && pop == COP_X && pn < 4096 && n < 65536) {
                out[len - 1] = (int32_t)((uint32_t)COP_XY | ((uint32_t)pn << 4) | ((uint32_t)n << 16));
                return;
            }
            if (op == COP_C1 && pop == COP_X) {
                out[len - 1] = (int32_t)(((uint32_t)pn << COP_SHIFT) | (uint32_t)COP_XC1);
                return;
            }
            if (op == COP_C2 && pop == COP_BX) {
                out[len - 1] = (int32_t)(((uint32_t)pn << COP_SHIFT) | (uint32_t)COP_BXC2);
                return;
            }
        }
        if (len >= cap) { ok = false; return; }
        out[len++] = (int32_t)(((uint32_t)n << COP_SHIFT) | (uint32_t)op);
    }
};

// one multi_row_sum stream of kk rows; ev_row/ev_q: this stream's events (rows increasing)
inline void emit_stream(CascEmitter& E, int kk, int lp, const int* ev_row, const int* ev_q,
                        int nev, int fin_reg) {
    const long L = 1L << lp, L2 = L * L, L3 = L2 * L;
    const long full = ((long)kk >> lp) << lp;
    int e = 0;
    auto next_ev = [&]() -> long { return e < nev ? (long)ev_row[e] : (1L << 40); };
    auto rows = [&](long r, long end) {        // rows [r, end) into a0
        while (r < end) {
            const long ne = next_ev();
            if (ne < end) {
                if (ne > r) E.put(COP_X, (int)(ne - r));
                E.put(COP_Y, ev_q[e]);
                ++e;
                r = ne + 1;
            } else {
                E.put(COP_X, (int)(end - r));
                r = end;
            }
        }
    };
    long i = 0;
    while (i < full) {
        if (i % L3 == 0 && i + L3 <= full && next_ev() >= i + L3) {
            int n = 0;
            while (i + L3 <= full && next_ev() >= i + L3) { ++n; i += L3; }
            E.put(COP_G2, n);
            continue;
        }
        if (i % L2 == 0 && i + L2 <= full && next_ev() >= i + L2) {
            int n = 0;
            do { ++n; i += L2; } while (i % L3 != 0 && i + L2 <= full && next_ev() >= i + L2);
            E.put(COP_G1, n);
            if (i % L3 == 0) E.put(COP_C3);
            continue;
        }
        if (next_ev() >= i + L) {                            // pure block(s)
            int n = 0;
            do { ++n; i += L; } while (i % L2 != 0 && i + L <= full && next_ev() >= i + L);
            E.put(COP_BX, n);
        } else {                                             // mixed block
            rows(i, i + L);
            E.put(COP_C1);
            i += L;
        }
        if (i % L2 == 0) {
            E.put(COP_C2);
            if (i % L3 == 0) E.put(COP_C3);
        }
    }
    rows(full, kk);
    E.put(COP_FIN, fin_reg);
}

inline int cascade_lp(long rows) {
    int c = 0;
    while ((1L << c) < rows) ++c;       // ceil_log2 (0 for rows <= 1)
    const int lp = c / 4;
    return lp < 4 ? 4 : lp;
}

inline int build_cascade_program(int k, const int32_t* pos, const int32_t* arr, int n_events,
                                 int32_t* prog, int cap, CascInfo* info) {
    if (k < 1 || k > CASC_MAX_K) return -3;
    for (int j = 0; j < n_events; ++j) {
        if (pos[j] < 0 || pos[j] >= k || arr[j] < 0 || arr[j] >= (1 << 26)) return -1;
        if (j && pos[j] <= pos[j - 1]) return -1;
    }
    const int lp = cascade_lp(k);
    if (cascade_lp(k / 4) != lp) return -3;
    CascEmitter E{prog, cap};
    // main program: multi_row_sum over all k entries
    {
        int* rows = new int[n_events > 0 ? n_events : 1];
        for (int j = 0; j < n_events; ++j) rows[j] = pos[j];
        emit_stream(E, k, lp, rows, arr, n_events, 0);
        E.put(COP_END);
        delete[] rows;
    }
    const int tail_off = E.len;
    E.stream_start = E.len;
    // row_sum program: 4 strided streams of k/4 rows, then the leftover rows into stream 0
    const int sz = k / 4;
    {
        int* rows = new int[n_events > 0 ? n_events : 1];
        int* qs = new int[n_events > 0 ? n_events : 1];
        for (int q = 0; q < 4; ++q) {
            int ne = 0;
            for (int j = 0; j < n_events; ++j)
                if (pos[j] % 4 == q && pos[j] / 4 < sz) { rows[ne] = pos[j] / 4; qs[ne++] = arr[j]; }
            emit_stream(E, sz, lp, rows, qs, ne, q);
        }
        int j = 0;
        while (j < n_events && pos[j] < 4 * sz) ++j;
        for (int p = 4 * sz; p < k; ++p) {
            if (j < n_events && pos[j] == p) E.put(COP_LY, arr[j++]);
            else E.put(COP_LX);
        }
        E.put(COP_RS);
        E.put(COP_END);
        delete[] rows;
        delete[] qs;
    }
    if (!E.ok || E.len + CASC_PAD - 1 > cap) return -2;
    for (int j = E.len; j < cap && j < E.len + CASC_PAD; ++j) prog[j] = COP_END;   // fetch pad
    if (info) *info = CascInfo{E.len, tail_off, E.need, lp};
    return E.len;
}

// ---- interpreter (host and device) -------------------------------------------------------------
// T = float (one element) or f32x4 (four elements in lock step); YF(q) returns entry array q's
// value(s); PROG indexes like a const int32_t* (uniform on the device: scalar loads).
template <class T>
struct CascVals {
    T x, bx, g1, g2;
};

template <class T>
__host__ __device__ inline T casc_seq_sum(T v, int n) {
    T a = T(0.f);
    for (int j = 0; j < n; ++j) a += v;
    return a;
}

template <class T>
__host__ __device__ inline CascVals<T> casc_values(T x, int need, int lp) {
    CascVals<T> c;
    c.x = x;
    c.bx = c.g1 = c.g2 = T(0.f);
    const int L = 1 << lp;
    if (need & 1) c.bx = casc_seq_sum(x, L);
    if (need & 2) c.g1 = casc_seq_sum(c.bx, L);
    if (need & 4) c.g2 = casc_seq_sum(c.g1, L);
    return c;
}

// a += v, n times in sequence (8-way unrolled body + fall-through remainder: one loop overhead
// per eight adds on the device)
template <class T>
__host__ __device__ inline void casc_add_n(T& a, const T& v, int n) {
    for (; n >= 8; n -= 8) {
        a += v;
        a += v;
        a += v;
        a += v;
        a += v;
        a += v;
        a += v;
        a += v;
    }
    switch (n) {
        case 7: a += v; [[fallthrough]];
        case 6: a += v; [[fallthrough]];
        case 5: a += v; [[fallthrough]];
        case 4: a += v; [[fallthrough]];
        case 3: a += v; [[fallthrough]];
        case 2: a += v; [[fallthrough]];
        case 1: a += v; [[fallthrough]];
        default: break;
    }
}

// FETCH words are read per step (the device passes CASC_PAD = 8: one wide scalar load per eight
// ops); the program buffer then needs FETCH - 1 readable words past its last COP_END.

// MAIN_ONLY: the caller runs main programs only (no row_sum part), so r1..r3 stay dead
template <int FETCH = 1, bool MAIN_ONLY = false, class T, class PROG, class YF>
__host__ __device__ inline T casc_run(const PROG& prog, int pc, const CascVals<T>& c, YF&& y) {
    T a0 = T(0.f), a1 = T(0.f), a2 = T(0.f), a3 = T(0.f);
    T r0 = T(0.f), r1 = T(0.f), r2 = T(0.f), r3 = T(0.f);
    for (;; pc += FETCH) {
        int32_t wv[FETCH];
#pragma unroll
        for (int k = 0; k < FETCH; ++k) wv[k] = prog[pc + k];
#pragma unroll
        for (int k = 0; k < FETCH; ++k) {
            const uint32_t w = (uint32_t)wv[k];
            const int op = (int)(w & 15u);
            const int n = (int)(w >> COP_SHIFT);
            // most frequent first: the event-block ops, then the group structure
            if (op == COP_XY) {
                casc_add_n(a0, c.x, n & 4095);
                a0 += y((int)(w >> 16));
            } else if (op == COP_X) {
                casc_add_n(a0, c.x, n);
            } else if (op == COP_XC1) {
                casc_add_n(a0, c.x, n);
                a1 += a0;
                a0 = T(0.f);
            } else if (op == COP_Y) {
                a0 += y(n);
            } else if (op == COP_BX) {
                casc_add_n(a1, c.bx, n);
            } else if (op == COP_BXC2) {
                casc_add_n(a1, c.bx, n);
                a2 += a1;
                a1 = T(0.f);
            } else if (op == COP_C1) {
                a1 += a0;
                a0 = T(0.f);
            } else if (op == COP_C2) {
                a2 += a1;
                a1 = T(0.f);
            } else if (op == COP_G1) {
                casc_add_n(a2, c.g1, n);
            } else if (op == COP_C3) {
                a3 += a2;
                a2 = T(0.f);
            } else if (op == COP_G2) {
                casc_add_n(a3, c.g2, n);
            } else if (op == COP_FIN) {
                T r = a0;
                r += a1;
                r += a2;
                r += a3;
                a0 = a1 = a2 = a3 = T(0.f);
                if (MAIN_ONLY || n == 0) r0 = r;
                else if (n == 1) r1 = r;
                else if (n == 2) r2 = r;
                else r3 = r;
            } else if (op == COP_LX) {
                r0 += c.x;
            } else if (op == COP_LY) {
                r0 += y(n);
            } else if (op == COP_RS) {
                if constexpr (!MAIN_ONLY) {
                    r0 += r1;
                    r0 += r2;
                    r0 += r3;
                }
            } else {
                return r0;      // COP_END
            }
        }
    }
}

}  // namespace flsim
