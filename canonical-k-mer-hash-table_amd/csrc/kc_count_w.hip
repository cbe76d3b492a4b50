// kc_count_w.hip -- the counting kernels and launchers for ONE key width: compiled once per
// W with -DKC_W=1..15 (k = 1..479: W = k / 32 + 1 u64 words per key), so the fifteen widths
// build as parallel translation units.  The kernels are kc_count_impl.h; kc_count.hip
// dispatches the C ABI's launch_* calls to WOps<W>.
#ifndef KC_W
#error "compile with -DKC_W=<key words>"
#endif
#include "kc_count_impl.h"

namespace kc {
template struct WOps<KC_W>;
}  // namespace kc
