// kc_compact_w.hip -- the compact-representation kernels (kc_compact_impl.h) for ONE key
// width: compiled once per W with -DKC_W=1..15, like kc_count_w.hip.
#ifndef KC_W
#error "compile with -DKC_W=<key words>"
#endif
#include "kc_internal.h"
#include "kc_compact_impl.h"

namespace kc {
template struct CompactOps<KC_W>;
}  // namespace kc
