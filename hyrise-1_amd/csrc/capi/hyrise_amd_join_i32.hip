// JoinHash host orchestration instantiated for hashed type int32_t (see join_host.hpp).
#include "join_host.hpp"

namespace hyj {
HYJ_DEFINE(i32, int32_t)
}  // namespace hyj
