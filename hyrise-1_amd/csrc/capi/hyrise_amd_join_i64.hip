// JoinHash host orchestration instantiated for hashed type int64_t (see join_host.hpp).
#include "join_host.hpp"

namespace hyj {
HYJ_DEFINE(i64, int64_t)
}  // namespace hyj
