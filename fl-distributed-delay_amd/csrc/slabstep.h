// Fused end of a server step (SURVEY 8 a6 + a8 + a9) over the weight-gradient slabs the networks'
// GEMMs accumulate during an epoch:
//
//   S_t = sum_z slab[z]                 agents.py:35 -- .grad accumulates over the epoch's workers
//   [S_out = S_t]                       main.py:156,161 -- the slow worker's FIFO entry (a tick)
//   g   = rule(weight_ups)              main.py:23-25  -- cascade mean over [S_t]*c + stale entries
//   Adam(p, m, v, g)                    agents.py:9-21 -- Central.update_model
//
// in ONE launch that streams every slab byte once.  A network describes its slabs as segments
// (one per parameter tensor: slab base, split count Z, slab row length n, where the tensor sits in
// the flat parameter vector, and the packed-conv layout that maps a slab column to torch's
// [co][ci][kh][kw]).  The planner cuts each segment into units of <= UNIT_FLOATS slab floats:
// 256 slab columns x a z-range.  A tile whose z-range is split over several units is finished by
// the unit that arrives last (counter per tile); its partials are handed over through sc1
// stores / loads (agent scope), the in-launch split-K recipe of cdna_hip_programming.md §5.
#pragma once
#include <stdint.h>

#include "cascade.h"
#include "common.h"
#include "flsim.h"

namespace flsim {

constexpr int STEP_MAX_SEG = 40;      // parameter tensors per network (vgg11_bn: 38)
constexpr int RULE_MAX_ARR = FLSIM_MAX_ARRAYS;   // weight_ups arrays besides S_t per launch
constexpr int RULE_INL_PROG = 192;    // program words carried in the kernel arguments
constexpr long STEP_UNIT_FLOATS = 65536;

// host description of one parameter tensor's gradient slabs (offsets in floats)
struct SegSpec {
    long slab_off;     // slab [Z][n] at gradstate + slab_off
    int Z;
    long n;
    long toff, numel;  // the tensor in the flat named_parameters vector
    int CO, CI, CIP, KP;   // packed conv layout n = CO * KP, column = co*KP + khkw*CIP + ci; CO = 0: identity
    int group = -1;        // slab-row group whose rows in use this epoch are tracked (-1: all Z)
};

// planned segment (kernel argument)
struct SlabSeg {
    long slab_off;
    int Z, n, zc, nz, tiles, tpu, unit0, tile0, toff, numel;
    uint16_t CO, CI, CIP, KP;
    uint16_t wide;   // identity layout, 16-B aligned, no row_sum tail: 1024-element float4 tiles
    int16_t group;   // SegSpec::group
    int zlim;        // rows [0, zlim) hold this epoch's sums (set per launch; the rest are stale)
};

struct StepPlan {
    SlabSeg seg[STEP_MAX_SEG];
    int nseg, units, ctiles;
    long slab_floats;     // sum of Z * n (the slab bytes the step streams / 4)
    int u_wide, u_conv;   // first unit of the wide (class 1) and packed conv (class 2) segments
};

// wide (float4) tiles: identity layout, 16-B aligned, no row_sum tail, a real weight matrix
inline bool seg_wide(const SegSpec& s) {
    return s.CO == 0 && s.n % 4 == 0 && s.toff % 4 == 0 && s.numel % 32 == 0 && s.n >= 4096;
}

// Dispatch order of the units: small tensors first (biases, the head, conv1: few units, each a
// long serial z-reduction), then the wide segments (the linear layers: many short units) and the
// packed conv segments (uniform 256 KB streaming units) interleaved in proportion (the kernel
// maps block positions onto the two runs), so the units that carry most of the rule() program's
// arithmetic (the linear layers' elements) run beside the ones that carry most of the slab bytes.
inline int seg_class(const SegSpec& s) { return s.n < 4096 ? 0 : (seg_wide(s) ? 1 : 2); }

inline int plan_step(const SegSpec* s_in, int nseg, StepPlan* P) {
    if (nseg > STEP_MAX_SEG) return 1;
    SegSpec s[STEP_MAX_SEG];
    int k = 0;
    for (int pass = 0; pass < 3; ++pass)
        for (int i = 0; i < nseg; ++i)
            if (seg_class(s_in[i]) == pass) s[k++] = s_in[i];
    P->nseg = nseg;
    int u = 0, ct = 0;
    long sf = 0;
    P->u_wide = P->u_conv = -1;
    for (int i = 0; i < nseg; ++i) {
        SlabSeg& g = P->seg[i];
        if (P->u_wide < 0 && seg_class(s[i]) >= 1) P->u_wide = u;
        if (P->u_conv < 0 && seg_class(s[i]) == 2) P->u_conv = u;
        g.slab_off = s[i].slab_off;
        g.Z = s[i].Z;
        g.n = (int)s[i].n;
        g.toff = (int)s[i].toff;
        g.numel = (int)s[i].numel;
        g.CO = (uint16_t)s[i].CO;
        g.CI = (uint16_t)s[i].CI;
        g.CIP = (uint16_t)s[i].CIP;
        g.KP = (uint16_t)s[i].KP;
        g.wide = seg_wide(s[i]);
        g.group = (int16_t)s[i].group;
        g.zlim = g.Z;
        g.tiles = (int)((s[i].n + (g.wide ? 1023 : 255)) / (g.wide ? 1024 : 256));
        const long tile_f = (g.wide ? 1024L : 256L) * s[i].Z;
        // wide tiles: 64 KB units (one tile of a few rows per block: many blocks in flight)
        const long unit_f = g.wide ? STEP_UNIT_FLOATS / 4 : STEP_UNIT_FLOATS;
        int units;
        if (tile_f <= unit_f) {
            g.nz = 1;
            g.zc = g.Z;
            long tpu = unit_f / tile_f;
            if (tpu > (g.wide ? 1 : 4)) tpu = g.wide ? 1 : 4;   // short units, no serial tails
            g.tpu = (int)(tpu < g.tiles ? tpu : g.tiles);
            units = (g.tiles + g.tpu - 1) / g.tpu;
            g.tile0 = 0;
        } else {
            int nz = (int)((tile_f + unit_f - 1) / unit_f);
            g.zc = (g.Z + nz - 1) / nz;
            g.zc = (g.zc + 3) / 4 * 4;
            g.nz = (g.Z + g.zc - 1) / g.zc;
            g.tpu = 1;
            units = g.tiles * g.nz;
            g.tile0 = ct;
            ct += g.tiles;
        }
        g.unit0 = u;
        u += units;
        sf += (long)s[i].Z * s[i].n;
    }
    P->units = u;
    if (P->u_wide < 0) P->u_wide = u;
    if (P->u_conv < 0) P->u_conv = u;
    P->ctiles = ct;
    P->slab_floats = sf;
    return 0;
}

// Adam hyper-parameters + rule() divisor, prepared on the host (agents.py:9-21, main.py:106)
struct AdamConst {
    float w1, b2, w2, bc2s, rbc2s, eps, neg_ss, fk, rk;
};

// rule(): which program and which arrays (host side, see flsim_rule in include/flsim.h)
struct RuleProg {
    const int32_t* prog;            // device program, or nullptr: iprog
    int32_t iprog[RULE_INL_PROG];
    CascInfo info;
    int narr;
    const float* arr[RULE_MAX_ARR]; // nullptr entry = zeros (torch-1.x stale semantics)
    int distinct;                   // distinct non-null arrays (algorithmic bytes)
};

// gradstate extras the fused step needs: tile counters (zeroed with the slabs) and partials
inline long step_counter_floats(const StepPlan& P) { return (P.ctiles + 63) / 64 * 64; }
inline long step_partial_floats(const StepPlan& P) { return (long)P.units * 1024; }

// launch: S_out (nullable) receives S_t in the flat layout; rule == nullptr: reduce only (the
// network's end_epoch); else rule() + Adam on p, m, v
int slab_step_launch(float* gradstate, const StepPlan& plan, long cnt_off, long part_off,
                     float* S_out, const RuleProg* rule, const AdamConst* ac, float* p, float* m,
                     float* v, long P, hipStream_t stream);

// host helpers shared with server.hip's C-ABI
int make_rule(const flsim_rule* r, RuleProg* out);
int make_adam_const(int divisor, long step, double lr, double beta1, double beta2, double eps,
                    AdamConst* ac);

}  // namespace flsim
