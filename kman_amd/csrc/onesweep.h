// onesweep.h — decoupled look-back pieces shared by the onesweep digit passes
// (sort.hip) and the region passes (region.hip).  Status words are
// flag:2 | epoch:6 | value:56 (common.h), RADIX per tile, digit-major inside.
#pragma once
#include "common.h"

namespace {

constexpr int RADIX = 256;
#ifndef KMAN_LB
#define KMAN_LB 8
#endif
constexpr int LB = KMAN_LB;  // predecessor status words fetched per look-back round


// publish a tile's digit count: inclusive for a chain's first tile
template <int STRIDE = RADIX>
KMAN_DEV void digit_publish(uint64_t *st, int64_t tile, int64_t first, uint64_t agg, uint32_t epoch) {
    st_store(&st[(uint64_t)tile * STRIDE], st_make(tile == first ? ST_INCL : ST_AGG, epoch, agg));
}

// TPD adjacent lanes walk one digit's chain together: lane `sub` of the group
// loads predecessors base - sub*LB - q (q < LB), so one round covers TPD*LB
// tiles.  With many tiles in flight the inclusive-prefix frontier lags by
// (look-back time / tile start interval) tiles, so the pass runs at about
// (predecessors per round) / (round latency) tiles per unit time: widening the
// round is what raises it.  The aggregate has been published already (EARLY).
// LBN: predecessors per lane per round (short chains whose predecessors are
// usually done: 1 or 2, so one round costs few status loads)
template <int TPD, int LBN = LB, int STRIDE = RADIX>
KMAN_DEV uint64_t group_lookback(uint64_t *st, int64_t tile, int64_t first, uint64_t agg, uint32_t epoch,
                                uint32_t *err) {
    const int lane = lane_id();
    const int sub = lane % TPD;
    const int g0 = lane - sub;
    if (tile == first) return 0;  // a chain's first tile published its inclusive count with the aggregate
    uint64_t excl = 0;
    int64_t base = tile - 1;
    uint32_t spins = 0;
    while (base >= first) {
        uint64_t w[LBN];
#pragma unroll
        for (int q = 0; q < LBN; q++) {
            const int64_t j = base - (int64_t)sub * LBN - q;
            w[q] = j >= first ? st_load(&st[(uint64_t)j * STRIDE]) : st_make(ST_INCL, epoch, 0);
        }
        // this lane's segment, in distance order: 0 all AGG, 1 met INCL, 2 stalled
        uint32_t state = 0, used = 0;
        uint64_t sum = 0;
#pragma unroll
        for (int q = 0; q < LBN; q++) {
            if (state) continue;
            const uint64_t f = st_flag(w[q], epoch);
            if (f == 0) {
                state = 2;
                continue;
            }
            sum += w[q] & ST_VMASK;
            used++;
            if (f == ST_INCL) state = 1;
        }
        // combine the group's segments in distance order
        const uint64_t m = (__ballot(state != 0) >> g0) & ((1ull << TPD) - 1);
        const int first = m ? __ffsll((unsigned long long)m) - 1 : TPD;
        uint64_t tot = 0;
        int64_t adv = 0;
#pragma unroll
        for (int s = 0; s < TPD; s++) {
            const uint64_t ss = shfl_any(sum, g0 + s);
            const uint32_t su = (uint32_t)__shfl((int)used, g0 + s, 64);
            if (s <= first) {
                tot += ss;
                adv += su;
            }
        }
        const uint32_t fstate = first < TPD ? (uint32_t)__shfl((int)state, g0 + first, 64) : 0;
        excl += tot;
        if (fstate == 1) break;
        base -= first < TPD ? adv : (int64_t)TPD * LBN;
        if (fstate == 2) {
            if (spin_give_up(spins, err, 2u)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (sub == 0) st_store(&st[(uint64_t)tile * STRIDE], st_make(ST_INCL, epoch, excl + agg));
    return excl;
}

}  // namespace
