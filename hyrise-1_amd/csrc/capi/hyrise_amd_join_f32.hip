// JoinHash host orchestration instantiated for hashed type float (see join_host.hpp).
#include "join_host.hpp"

namespace hyj {
HYJ_DEFINE(f32, float)
}  // namespace hyj
