// Internal declarations shared by the convolution (conv.hip) and weight-gradient (wgrad.hip) units.
#pragma once
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

namespace hyres {

constexpr int KT = 32;  // K chunk (floats)

// tile / split-K overrides set through hyres_conv_tuning (conv.hip; -1 = the planners' heuristics)
extern int g_tune[8];

}  // namespace hyres
