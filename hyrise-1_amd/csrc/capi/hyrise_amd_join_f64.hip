// JoinHash host orchestration instantiated for hashed type double (see join_host.hpp).
#include "join_host.hpp"

namespace hyj {
HYJ_DEFINE(f64, double)
}  // namespace hyj
