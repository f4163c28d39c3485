// Trunk kernels with 128 filters (trunk_variants.h).
#include "trunk_variants.h"

namespace gznn {

KernelChoice trunk_variant_f128(int pt, int v, int precision) {
    switch (pt) {
        case 2: return variants<128, 2>(v, precision);
        case 3: return variants<128, 3>(v, precision);
        case 4: return variants<128, 4>(v, precision);
        case 5: return variants<128, 5>(v, precision);
        case 6: return variants<128, 6>(v, precision);
        case 7: return variants<128, 7>(v, precision);
        case 8: return variants<128, 8>(v, precision);
        case 9: return variants<128, 9>(v, precision);
        case 10: return variants<128, 10>(v, precision);
        case 11: return variants<128, 11>(v, precision);
        case 23: return variants<128, 23>(v, precision);   // 19 x 19
        default: return KernelChoice{};
    }
}

}  // namespace gznn
