// tonemap.cpp -- exact gamma/quantise table for the device epilogue.
//
// The reference quantises with `round(255 * std::pow(x, (float)(1./2.2)))`
// (/root/reference/hw5/src/color.cpp:37-48): glibc powf, not correctly
// rounded.  Instead of restating powf on the device, the host (same libm as
// the reference's CPU run) computes, for every 8-bit level k = 1..255, the
// smallest float v in [0, 1] whose quantised value is >= k.  The device maps
// a saturated channel value to (number of thresholds <= v), which equals the
// reference's byte whenever the host map is monotone in v -- checked
// exhaustively over all 1,065,353,217 floats in [0, 1] by
// tests/test_host.py::test_gamma_table_monotone (slow test).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "pt_scene.h"

namespace pth {
namespace {
inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
inline int quant(float v) {
    const float g = (float)(1. / 2.2);
    return (int)round((double)(255.f * powf(v, g)));
}
}  // namespace

void build_gamma_thresholds(float thr[256]) {
    for (int k = 1; k <= 255; ++k) {
        uint32_t lo = 0u, hi = 0x3f800000u;  // q(bits(hi)) = 255 >= k
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2u;
            if (quant(bits_f(mid)) >= k) hi = mid; else lo = mid + 1u;
        }
        thr[k - 1] = bits_f(lo);
    }
    thr[255] = INFINITY;
}

}  // namespace pth
