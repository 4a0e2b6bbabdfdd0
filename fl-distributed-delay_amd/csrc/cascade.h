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

// Keeps a conditional block a real (uniform, scalar) branch: without it the compiler speculates a
// short run of adds and picks the result with v_cndmask, which executes every add of both paths
// (lab: 2.7x the VALU instructions of the program's adds, tools/lab/casc_lab.hip).
template <class T>
__host__ __device__ inline void casc_pin(T& a) {
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr (sizeof(T) == 4) {
        asm volatile("" : "+v"(a));
    } else {
        typedef float f4 __attribute__((ext_vector_type(4)));
        constexpr int W = sizeof(T) / 16;
        f4* q = reinterpret_cast<f4*>(&a);
#pragma unroll
        for (int i = 0; i < W; ++i) asm volatile("" : "+v"(q[i]));
    }
#else
    (void)a;
#endif
}

// a += v, n times in sequence.  n is uniform; its binary digits pick straight-line runs of 8, 4, 2
// and 1 adds (all the adds are the same operation, so their grouping does not change the result):
// four scalar bit tests and no loop for the n < 16 of every block-level word.
template <class T>
__host__ __device__ inline void casc_add_n(T& a, const T& v, int n) {
    if (n >= 32) {                      // only G2 runs of very large k
        for (; n >= 16; n -= 16) {
#pragma unroll
            for (int j = 0; j < 16; ++j) a += v;
        }
        casc_pin(a);
    }
    if (n & 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) a += v;
        casc_pin(a);
    }
    if (n & 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a += v;
        casc_pin(a);
    }
    if (n & 4) {
        a += v;
        a += v;
        a += v;
        a += v;
        casc_pin(a);
    }
    if (n & 2) {
        a += v;
        a += v;
        casc_pin(a);
    }
    if (n & 1) {
        a += v;
        casc_pin(a);
    }
}

// FETCH words are read per step; the program buffer then needs FETCH readable words past its last
// COP_END (CASC_PAD).  FETCH = 1 is the device form: one word executes while the next one's scalar
// load is in flight, and the interpreter body exists once.  Unrolling the body FETCH times (one
// wide scalar load per FETCH ops) made the general-order server step 115 KB of code, larger than
// the instruction cache, and every op then waited on an instruction fetch.

// MAIN_ONLY: the caller runs main programs only (no row_sum part), so r1..r3 stay dead
template <int FETCH = 1, bool MAIN_ONLY = false, class T, class PROG, class YF>
__host__ __device__ inline T casc_run(const PROG& prog, int pc, const CascVals<T>& c, YF&& y) {
    T a0 = T(0.f), a1 = T(0.f), a2 = T(0.f), a3 = T(0.f);
    T r0 = T(0.f), r1 = T(0.f), r2 = T(0.f), r3 = T(0.f);
    int32_t wv[FETCH];
#pragma unroll
    for (int k = 0; k < FETCH; ++k) wv[k] = prog[pc + k];
    for (;;) {
        pc += FETCH;
        int32_t wn[FETCH];                       // the next step's words, loaded ahead
#pragma unroll
        for (int k = 0; k < FETCH; ++k) wn[k] = prog[pc + k];
#pragma unroll
        for (int k = 0; k < FETCH; ++k) {
            const uint32_t w = (uint32_t)wv[k];
            const int op = (int)(w & 15u);
            const int n = (int)(w >> COP_SHIFT);
            switch (op) {
                case COP_XY:
                    casc_add_n(a0, c.x, n & 4095);
                    a0 += y((int)(w >> 16));
                    break;
                case COP_X:
                    casc_add_n(a0, c.x, n);
                    break;
                case COP_XC1:
                    casc_add_n(a0, c.x, n);
                    a1 += a0;
                    a0 = T(0.f);
                    break;
                case COP_Y:
                    a0 += y(n);
                    break;
                case COP_BX:
                    casc_add_n(a1, c.bx, n);
                    break;
                case COP_BXC2:
                    casc_add_n(a1, c.bx, n);
                    a2 += a1;
                    a1 = T(0.f);
                    break;
                case COP_C1:
                    a1 += a0;
                    a0 = T(0.f);
                    break;
                case COP_C2:
                    a2 += a1;
                    a1 = T(0.f);
                    break;
                case COP_G1:
                    casc_add_n(a2, c.g1, n);
                    break;
                case COP_C3:
                    a3 += a2;
                    a2 = T(0.f);
                    break;
                case COP_G2:
                    casc_add_n(a3, c.g2, n);
                    break;
                case COP_FIN: {
                    T r = a0;
                    r += a1;
                    r += a2;
                    r += a3;
                    a0 = a1 = a2 = a3 = T(0.f);
                    if (MAIN_ONLY || n == 0) r0 = r;
                    else if (n == 1) r1 = r;
                    else if (n == 2) r2 = r;
                    else r3 = r;
                    break;
                }
                case COP_LX:
                    r0 += c.x;
                    break;
                case COP_LY:
                    r0 += y(n);
                    break;
                case COP_RS:
                    if constexpr (!MAIN_ONLY) {
                        r0 += r1;
                        r0 += r2;
                        r0 += r3;
                    }
                    break;
                default:
                    return r0;      // COP_END
            }
        }
#pragma unroll
        for (int k = 0; k < FETCH; ++k) wv[k] = wn[k];
    }
}

// ---- macro words: the device form of a program ---------------------------------------------------
// One 64-bit macro word carries a whole stretch of ops in the fixed section order
//   lo: [x-run a0] [y_q into a0] [x-run a0] [C1] [bx-run a1] [C2] [g1-run a2] [C3]
//   hi: [g2-run a3] [FIN r] [LX | LY q] [RS] [END]
// (any section may be empty), so one stale entry -- the rest of its block, its level-1 group and
// its level-2 group -- is usually ONE word instead of 3-5 ops.  The interpreter body is a straight
// chain of uniform tests on the word's fields (no multiway dispatch): fewer loop trips, fewer
// scalar instructions per element, and a control flow the compiler keeps free of register copies.
// The packer keeps the op order exactly (it only groups consecutive ops into words), so a macro
// program computes the same roundings as its op program (tests/test_cascade_program.py).
constexpr uint32_t MW_Y = 1u << 5, MW_C1 = 1u << 17, MW_C2 = 1u << 23, MW_C3 = 1u << 29;
constexpr uint32_t MH_FIN = 1u << 16, MH_LX = 1u << 19, MH_LY = 1u << 20, MH_RS = 1u << 27,
                   MH_END = 1u << 28;
constexpr int MW_RUN_MAX = 31;          // x / bx / g1 runs per field (5 bits)

struct MacroPacker {
    uint32_t* out;        // pairs (lo, hi)
    int cap, len = 0;     // in pairs
    bool ok = true;
    uint32_t lo = 0, hi = 0;
    int cur = -1;         // last section used in the open word
    void flush() {
        if (cur < 0) return;
        if (len >= cap) { ok = false; return; }
        out[2 * len] = lo;
        out[2 * len + 1] = hi;
        ++len;
        lo = hi = 0;
        cur = -1;
    }
    // section s (0..12) of the open word, or a new word when s does not come after `cur`
    void at(int s) {
        if (s <= cur) flush();
        cur = s;
    }
    // a run of n adds into one accumulator: x runs may sit in section 0 (bits 0-4) or 2 (bits
    // 12-16), bx runs in 4 (18-22), g1 runs in 6 (24-28); a run right after the same kind of run
    // extends it (consecutive runs of one op are the same adds)
    void run(int s0, int s1, int sh0, int n) {
        while (n > 0) {
            if (cur >= 0 && (cur == s0 || cur == s1)) {
                const int sh = cur == s0 ? sh0 : 12;
                const int have = (int)((lo >> sh) & 31u);
                const int add = n < MW_RUN_MAX - have ? n : MW_RUN_MAX - have;
                if (add > 0) {
                    lo += (uint32_t)add << sh;
                    n -= add;
                    continue;
                }
            }
            int s = s0, sh = sh0;
            if (s0 <= cur) {
                if (s1 > cur) {
                    s = s1;
                    sh = 12;
                } else {
                    flush();
                }
            }
            cur = s;
            const int add = n < MW_RUN_MAX ? n : MW_RUN_MAX;
            lo |= (uint32_t)add << sh;
            n -= add;
        }
    }
    void op(uint32_t w) {
        const int o = (int)(w & 15u);
        int n = (int)(w >> COP_SHIFT);
        switch (o) {
            case COP_X: run(0, 2, 0, n); break;
            case COP_XY: run(0, 2, 0, n & 4095); y((int)(w >> 16)); break;
            case COP_XC1: run(0, 2, 0, n); at(3); lo |= MW_C1; break;
            case COP_Y: y(n); break;
            case COP_C1: at(3); lo |= MW_C1; break;
            case COP_BX: run(4, -1, 18, n); break;
            case COP_BXC2: run(4, -1, 18, n); at(5); lo |= MW_C2; break;
            case COP_C2: at(5); lo |= MW_C2; break;
            case COP_G1: run(6, -1, 24, n); break;
            case COP_C3: at(7); lo |= MW_C3; break;
            case COP_G2:
                for (; n > 0;) {
                    if (cur != 8) at(8);
                    const int have = (int)(hi & 0xffffu);
                    const int add = n < 0xffff - have ? n : 0xffff - have;
                    if (add == 0) { flush(); continue; }
                    hi += (uint32_t)add;
                    n -= add;
                }
                break;
            case COP_FIN: at(9); hi |= MH_FIN | ((uint32_t)(n & 3) << 17); break;
            case COP_LX: at(10); hi |= MH_LX; break;
            case COP_LY: at(10); hi |= MH_LY | ((uint32_t)(n & 63) << 21); break;
            case COP_RS: at(11); hi |= MH_RS; break;
            default: at(12); hi |= MH_END; break;
        }
    }
    void y(int q) {
        at(1);
        lo |= MW_Y | ((uint32_t)(q & 63) << 6);
    }
};

// ops from prog[start] through its COP_END -> macro pairs appended to P; returns false on overflow
// or an array index past 63 (the macro form's limit, RULE_MAX_ARR)
inline bool pack_macro(const int32_t* prog, int start, MacroPacker& P) {
    for (int pc = start;; ++pc) {
        const uint32_t w = (uint32_t)prog[pc];
        const int o = (int)(w & 15u);
        if ((o == COP_Y || o == COP_LY) && (w >> COP_SHIFT) > 63) return false;
        if (o == COP_XY && (w >> 16) > 63) return false;
        P.op(w);
        if (o == COP_END) break;
    }
    P.flush();
    return P.ok;
}

// a whole program (main + row_sum part) as macro pairs: out[2 * cap] words; minfo = {pairs, pair
// index of the row_sum part, need, lp}.  Returns the pair count or a negative error.
inline int build_macro_program(const int32_t* prog, const CascInfo& info, uint32_t* out, int cap,
                               CascInfo* minfo) {
    MacroPacker P{out, cap};
    if (!pack_macro(prog, 0, P)) return -2;
    const int tail = P.len;
    if (!pack_macro(prog, info.tail_off, P)) return -2;
    // fetch pad: the interpreter loads the next pair while it runs the END pair
    if (P.len + 1 > cap) return -2;
    out[2 * P.len] = 0;
    out[2 * P.len + 1] = MH_END;
    if (minfo) *minfo = CascInfo{P.len, tail, info.need, info.lp};
    return P.len;
}

// a += v, n times, 1 <= n <= 31 (bits of a uniform n, each run a pinned branch)
template <class T>
__host__ __device__ inline void casc_run5(T& a, const T& v, uint32_t n) {
    if (n & 16u) {
#pragma unroll
        for (int j = 0; j < 16; ++j) a += v;
        casc_pin(a);
    }
    if (n & 8u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a += v;
        casc_pin(a);
    }
    if (n & 4u) {
        a += v;
        a += v;
        a += v;
        a += v;
        casc_pin(a);
    }
    if (n & 2u) {
        a += v;
        a += v;
        casc_pin(a);
    }
    if (n & 1u) {
        a += v;
        casc_pin(a);
    }
}

// PROG2 indexes pairs: prog.lo(i), prog.hi(i) (uniform scalar loads on the device)
template <bool MAIN_ONLY = false, class T, class PROG2, class YF>
__host__ __device__ inline T casc_run_macro(const PROG2& prog, int pc, const CascVals<T>& c,
                                            YF&& y) {
    T a0 = T(0.f), a1 = T(0.f), a2 = T(0.f), a3 = T(0.f);
    T r0 = T(0.f), r1 = T(0.f), r2 = T(0.f), r3 = T(0.f);
    uint32_t lo = prog.lo(pc), hi = prog.hi(pc);
    for (;;) {
        ++pc;
        const uint32_t nlo = prog.lo(pc), nhi = prog.hi(pc);     // the next pair, loaded ahead
        if (lo) {
            uint32_t n = lo & 31u;
            if (n) casc_run5(a0, c.x, n);
            if (lo & MW_Y) {
                a0 += y((int)((lo >> 6) & 63u));
                casc_pin(a0);
            }
            n = (lo >> 12) & 31u;
            if (n) casc_run5(a0, c.x, n);
            if (lo & MW_C1) {
                a1 += a0;
                a0 = T(0.f);
                casc_pin(a1);
            }
            n = (lo >> 18) & 31u;
            if (n) casc_run5(a1, c.bx, n);
            if (lo & MW_C2) {
                a2 += a1;
                a1 = T(0.f);
                casc_pin(a2);
            }
            n = (lo >> 24) & 31u;
            if (n) casc_run5(a2, c.g1, n);
            if (lo & MW_C3) {
                a3 += a2;
                a2 = T(0.f);
                casc_pin(a3);
            }
        }
        if (hi) {
            const int n = (int)(hi & 0xffffu);
            if (n) casc_add_n(a3, c.g2, n);
            if (hi & MH_FIN) {
                T r = a0;
                r += a1;
                r += a2;
                r += a3;
                a0 = a1 = a2 = a3 = T(0.f);
                const uint32_t reg = (hi >> 17) & 3u;
                if (MAIN_ONLY || reg == 0) r0 = r;
                else if (reg == 1) r1 = r;
                else if (reg == 2) r2 = r;
                else r3 = r;
            }
            if (hi & MH_LX) r0 += c.x;
            if (hi & MH_LY) r0 += y((int)((hi >> 21) & 63u));
            if (hi & MH_RS) {
                if constexpr (!MAIN_ONLY) {
                    r0 += r1;
                    r0 += r2;
                    r0 += r3;
                }
            }
            if (hi & MH_END) return r0;
        }
        lo = nlo;
        hi = nhi;
    }
}

}  // namespace flsim
