// Trunk kernels with 64 filters, v2 (pre-activation / squeeze-excite) nets (trunk_variants.h).
#include "trunk_variants.h"

namespace gznn {

KernelChoice trunk_variant_f64_v2(int pt, int v, int precision) {
    switch (pt) {
        case 2: return variants<64, 2, true>(v, precision);
        case 3: return variants<64, 3, true>(v, precision);
        case 4: return variants<64, 4, true>(v, precision);
        case 5: return variants<64, 5, true>(v, precision);
        case 6: return variants<64, 6, true>(v, precision);
        case 7: return variants<64, 7, true>(v, precision);
        case 8: return variants<64, 8, true>(v, precision);
        case 9: return variants<64, 9, true>(v, precision);
        case 10: return variants<64, 10, true>(v, precision);
        case 11: return variants<64, 11, true>(v, precision);
        default: return KernelChoice{};
    }
}

}  // namespace gznn
