// Static instruction counts of each step kind of the path engine's query
// (pt_query.h q_exec), one kernel per kind with the kind fixed so that the
// compiler keeps only that branch:  hipcc -S, then tools/micro/qexec_sizes.py.
// Diagnostics only (not part of the library).
#include <hip/hip_runtime.h>

#include "pt_devutil.h"
#include "pt_query.h"

using namespace pt;

template <int K>
__global__ void __launch_bounds__(64) k_kind(SceneView S, Query* qs, const F4* rs, QCounts* cs, uint32_t* stk_g) {
    __shared__ uint32_t stk[17 * 64];
    const uint32_t i = threadIdx.x;
    Query q = qs[i];
    F4 r[8];
    for (int k = 0; k < 8; ++k) r[k] = rs[8 * i + k];
    if (K == 0) { q.phase = Q_AUX; q.node &= 0x7fffffffu; }             // aux node
    if (K == 1) { q.phase = Q_AUX; q.node |= PT_LEAFQ; }                 // probe
    if (K == 2) { q.phase = Q_REPLAY; q.walk = R_CAND; }                 // leaf check
    if (K == 3) { q.phase = Q_REPLAY; q.walk = R_WALK_E; }               // walk entries
    if (K == 4) { q.phase = Q_REPLAY; q.walk = R_WALK_N; }               // walk nodes
    LdsMemN<64u> m{stk + i, stk_g[0], 16u};
    QCounts C = cs[i];
    q_exec(S, q, C, m, r);
    qs[i] = q;
    cs[i] = C;
}
template __global__ void k_kind<0>(SceneView, Query*, const F4*, QCounts*, uint32_t*);
template __global__ void k_kind<1>(SceneView, Query*, const F4*, QCounts*, uint32_t*);
template __global__ void k_kind<2>(SceneView, Query*, const F4*, QCounts*, uint32_t*);
template __global__ void k_kind<3>(SceneView, Query*, const F4*, QCounts*, uint32_t*);
template __global__ void k_kind<4>(SceneView, Query*, const F4*, QCounts*, uint32_t*);
