// Trunk kernels with 256 filters (trunk_variants.h).
#include "trunk_variants.h"

namespace gznn {

KernelChoice trunk_variant_f256(int pt, int v, int precision) {
    switch (pt) {
        case 4: return variants<256, 4>(v, precision);
        case 7: return variants<256, 7>(v, precision);
        case 11: return variants<256, 11>(v, precision);
        default: return KernelChoice{};
    }
}

}  // namespace gznn
