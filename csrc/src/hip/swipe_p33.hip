// P33-letter instances of the swipe kernel (host streams: final's GPU slices and the headline bench read
// their letters as 7-letter 33-bit fields over PCIe); the template and the host side are in swipe_impl.hpp
// and swipe_kernels.hip.
#include "swipe_impl.hpp"

namespace moc {
namespace dev {

bool launch_swipe_p33(const ProblemView& pv, const ShortArgs& b, const SwipeLayout& lay, dim3 grid, dim3 block,
                      hipStream_t stream) {
  return launch_swipe_form<2>(pv, b, lay, grid, block, stream);
}

void preload_swipe_p33_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&swipe_search_kernel<24, 4, 2, false>));
}

}  // namespace dev
}  // namespace moc
