// Trunk kernels with 64 filters (trunk_variants.h).
#include "trunk_variants.h"

namespace gznn {

KernelChoice trunk_variant_f64(int pt, int v, int precision) {
    switch (pt) {
        case 2: return variants<64, 2>(v, precision);
        case 3: return variants<64, 3>(v, precision);
        case 4: return variants<64, 4>(v, precision);
        case 5: return variants<64, 5>(v, precision);
        case 6: return variants<64, 6>(v, precision);
        case 7: return variants<64, 7>(v, precision);
        case 8: return variants<64, 8>(v, precision);
        case 9: return variants<64, 9>(v, precision);
        case 10: return variants<64, 10>(v, precision);
        case 11: return variants<64, 11>(v, precision);
        default: return KernelChoice{};
    }
}

}  // namespace gznn
