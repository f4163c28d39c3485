// State -> input planes.  Restates GdlBasesTransformer (reference src/cpp/gdltransformer.h:69-149,
// gdltransformer.cpp:22-52): board bases set a single 1.0 at a precomputed buffer offset
// (channel_id*channel_size + y_idx*num_rows + x_idx, cppinterface.py:44), control bases flood-fill
// their channel with a value; planes are float32 channels-first [C][H][W].
#pragma once

#include <cstdint>
#include <set>
#include <vector>

namespace gz {

class GdlBasesTransformer {
public:
    GdlBasesTransformer(int channel_size, int channels_per_state, int num_control_channels,
                        int num_prev_states, int num_rewards, std::vector<int> expected_policy_sizes)
        : channel_size(channel_size), channels_per_state(channels_per_state),
          num_control_channels(num_control_channels), num_prev_states(num_prev_states),
          num_rewards(num_rewards), expected_policy_sizes(std::move(expected_policy_sizes)) {}

    void addBoardBase(int base_indx, int buf_incr) {
        board_space.push_back({base_indx, buf_incr});
        interested.insert(base_indx);
        if ((int)board_offset.size() <= base_indx) board_offset.resize(base_indx + 1, -1);
        board_offset[base_indx] = buf_incr;
    }
    void addControlBase(int base_indx, int channel_id, float value) {
        control_space.push_back({base_indx, channel_id, value});
        interested.insert(base_indx);
    }

    int totalSize() const {
        return channel_size * (channels_per_state * (num_prev_states + 1) + num_control_channels);
    }
    int getNumberPrevStates() const { return num_prev_states; }
    int getNumberPolicies() const { return (int)expected_policy_sizes.size(); }
    int getPolicySize(int i) const { return expected_policy_sizes[i]; }
    int getNumberRewards() const { return num_rewards; }
    int getChannelSize() const { return channel_size; }

    // gdltransformer.cpp:22-52, including the reference quirk that the previous-state slot index
    // `count` is never advanced (all previous states land in slot 1; identical for
    // num_previous_states <= 1, the only setting the BASELINE configs use).
    void toChannels(const uint64_t* state, const std::vector<const uint64_t*>& prev_states, float* buf) const;

    // Mask of the bases the transformer reads (gdltransformer.cpp:54-63): the key of the
    // duplicate-state and transposition maps.
    std::vector<uint64_t> createHashMask(int num_bases) const;

private:
    struct BoardBase { int base_indx, buf_incr; };
    struct ControlBase { int base_indx, channel_id; float value; };

    void setForState(float* local_buf, const uint64_t* bs) const;
    int controlStatesStart() const { return channel_size * (channels_per_state * (num_prev_states + 1)); }

    const int channel_size, channels_per_state, num_control_channels, num_prev_states, num_rewards;
    std::vector<int> expected_policy_sizes;
    std::vector<BoardBase> board_space;
    std::vector<int> board_offset;     // base index -> buffer offset (-1: not a board base)
    std::vector<ControlBase> control_space;
    std::set<int> interested;
};

}  // namespace gz
