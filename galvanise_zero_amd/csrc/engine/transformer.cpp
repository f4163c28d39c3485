#include "transformer.h"

#include "sm.h"

#include <cstring>

namespace gz {

void GdlBasesTransformer::setForState(float* local_buf, const uint64_t* bs) const {
    // same result as testing every board base in turn (gdltransformer.cpp:14-20): visit set bits only
    const int nbits = (int)board_offset.size();
    for (int w = 0; w * 64 < nbits; ++w) {
        uint64_t word = bs[w];
        while (word) {
            const int i = __builtin_ctzll(word) + 64 * w;
            word &= word - 1;
            if (i < nbits && board_offset[i] >= 0) local_buf[board_offset[i]] = 1.0f;
        }
    }
}

void GdlBasesTransformer::toChannels(const uint64_t* state, const std::vector<const uint64_t*>& prev_states,
                                     float* buf) const {
    std::memset(buf, 0, sizeof(float) * totalSize());
    setForState(buf, state);

    const int count = 1;   // never incremented in the reference (gdltransformer.cpp:38-43)
    for (const uint64_t* b : prev_states) setForState(buf + channels_per_state * channel_size * count, b);

    float* control_buf_start = buf + controlStatesStart();
    for (const ControlBase& c : control_space) {
        if (bs_get(state, c.base_indx)) {
            float* p = control_buf_start + channel_size * c.channel_id;
            for (int i = 0; i < channel_size; ++i) p[i] = c.value;
        }
    }
}

std::vector<uint64_t> GdlBasesTransformer::createHashMask(int num_bases) const {
    std::vector<uint64_t> mask((num_bases + 63) / 64, 0);
    for (int i : interested)
        if (i < num_bases) bs_set(mask.data(), i, true);
    return mask;
}

}  // namespace gz
