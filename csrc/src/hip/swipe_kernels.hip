// Inter-record swipe kernel: host-side configuration, dispatch and launch. The kernel template and its
// derivation are in swipe_impl.hpp; its instances in one code object per (letter form, NOFF),
// swipe_group.inc.
#include "swipe_impl.hpp"

namespace moc {
namespace dev {

namespace {
struct SwipeChoice {
  int noff = 0, l2w = 0;
  bool rk = false;
};

// Offsets per lane (NOFF), record words (L2W) and key form for a batch, or noff 0 when the kernel cannot
// take it: at most 64 offsets and 128 letters per record, the profile within the LDS budget, and an
// int16-exact key form (moc/kernel_bounds.hpp swipe_keys: the keys carry k when 2^KB * |D| leaves room, as
// on input6; otherwise, input1's W1 = 100, the RK form re-finds k after the selection).
// Offsets per lane: the batch's widest record offset range under its semantics (swipe_offsets; the
// reference's needs one offset less than lanes_needed), rounded up to a multiple of 4 (one ds_read_b64 per 4
// offsets, the epilogue's groups of 4): input6 / input1 run 20 offsets per lane instead of 24.
SwipeChoice swipe_choice(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t max_abs_weight, bool spec) {
  SwipeChoice c;
  const int64_t mn = std::min(min_l2, L1);
  if (lanes_needed(L1, mn) > 64 || max_l2 > bounds::kSwipeMaxL2) return c;
  const bounds::SwipeKeys keys = bounds::swipe_keys(max_abs_weight, max_l2);
  if (keys == bounds::SwipeKeys::None) return c;
  c.rk = keys == bounds::SwipeKeys::RK;
  c.noff = static_cast<int>(((std::max<int64_t>(swipe_offsets(L1, mn, spec), 4) + 3) / 4) * 4);
  c.l2w = bounds::swipe_record_words(max_l2);
  return c;
}
}  // namespace

int32_t swipe_form(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t max_abs_weight) {
  const SwipeChoice ch = swipe_choice(L1, min_l2, max_l2, max_abs_weight, true);
  return !ch.noff ? 0 : ch.rk ? bounds::kFormSwipeRK : bounds::kFormSwipeKBits;
}

bool configure_swipe(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t max_abs_weight, ShortArgs& a, bool hbm,
                     bool spec) {
  if (a.packed5) return false;  // 5-bit letters go through the staged pipeline (unpacked on the device)
  const SwipeChoice ch = swipe_choice(L1, min_l2, max_l2, max_abs_weight, spec);
  if (!ch.noff) return false;
  const int fb = result_bytes(static_cast<ResultFormat>(a.fmt));
  // host streams: 2048-record tiles (packed letters fit the register prefetch; 3.59 vs 3.69 ms per headline
  // step at 1024), device-resident: 512 (more blocks per CU); MOC_SWIPE_TILE overrides (64..2048)
  const int lf = letter_form(a);
  const int tile_cap = 256 * rpt_of(lf);
  int max_tile = std::min(hbm ? 512 : kMaxTile, tile_cap);
  if (const char* v = std::getenv("MOC_SWIPE_TILE")) max_tile = std::max(64, std::min(tile_cap, std::atoi(v)));
  for (int tr = max_tile; tr >= 64; tr /= 2) {
    const int cap = tr * static_cast<int>(std::max<int64_t>(max_l2, 1)) + 64;
    // a tile's letter bytes must fit the register prefetch (P33: 33 bits per 7 letters)
    if ((lf == 2 ? raw_cap(lf, cap) : cap + 32) > kMaxV * kBlock * 16) continue;
    SwipeLayout l = swipe_layout(static_cast<int>(L1), ch.noff, ch.l2w, tr, cap, fb, lf);
    if (l.total <= kLdsBudget) {
      a.tile_records = tr;
      a.codes_cap = cap;
      a.max_l2 = static_cast<int32_t>(max_l2);
      a.slot = ch.noff;  // offsets per lane
      a.rpw = ch.l2w;    // record words per lane
      a.swipe_rk = ch.rk ? 1 : 0;
      return true;
    }
  }
  return false;
}

#define MOC_SWIPE_PRELOAD_CALL(LF, NO) MOC_SWIPE_PRELOAD_FN(LF, NO)();
void preload_swipe_byte_kernels() { MOC_SWIPE_FOR_NOFF(MOC_SWIPE_PRELOAD_CALL, 0) }
void preload_swipe_p33_kernels() { MOC_SWIPE_FOR_NOFF(MOC_SWIPE_PRELOAD_CALL, 2) }
#undef MOC_SWIPE_PRELOAD_CALL

namespace {
// the instance's code object by letter form (0 bytes, 2 P33) and offsets per lane (a.slot)
bool launch_swipe_instance(int lf, const ProblemView& pv, const ShortArgs& b, const SwipeLayout& lay, dim3 grid,
                           dim3 block, int num_cus, hipStream_t stream) {
#define MOC_SWIPE_GROUP_CASE(LF, NO) \
  if (lf == LF && b.slot == NO) return MOC_SWIPE_FN(LF, NO)(pv, b, lay, grid, block, num_cus, stream);
  MOC_SWIPE_FOR_NOFF(MOC_SWIPE_GROUP_CASE, 0)
  MOC_SWIPE_FOR_NOFF(MOC_SWIPE_GROUP_CASE, 2)
#undef MOC_SWIPE_GROUP_CASE
  return false;
}
}  // namespace

// MOC_SWIPE_TAIL=0 keeps every tile at full size (A/B); 2, 4 (default), 8 or 16 cut the tail tiles to that
// fraction of a tile. Powers of two only: tiles stay multiples of 64 records (sparse-offset boundaries).
static int tail_div() {
  static const int d = [] {
    const char* v = std::getenv("MOC_SWIPE_TAIL");
    if (!v) return 4;
    const int x = std::atoi(v);
    return (x == 0 || x == 2 || x == 4 || x == 8 || x == 16) ? x : 4;
  }();
  return d;
}

void launch_swipe(const ProblemView& pv, const ShortArgs& a, int num_cus, hipStream_t stream) {
  if (a.n <= 0) return;
  const int fb = result_bytes(static_cast<ResultFormat>(a.fmt));
  if (a.lane_direct) {  // device-resident batches: the wave-autonomous kernel, LDS tables (+ P33 wave slices)
    if (a.off_shift > 6 || (a.off_shift && !(a.lengths3 || a.lengths4 || a.lengths6 || a.lengths8)) ||
        (!a.packed33 && a.off_shift) || (a.packed33 && a.rpw > 16))
      throw Error("launch_swipe: lane-direct batches are byte letters with dense offsets, or P33 letters with "
                  "64-record sparse offsets and lengths");
    const int lf = letter_form(a);
    const SwipeLayout lay = direct_layout(pv.L1, a.slot, a.rpw, lf, a.max_l2);
    if (!launch_swipe_instance(lf, pv, a, lay, dim3(1), dim3(kBlockD), num_cus, stream))
      throw Error("launch_swipe: no instance for this configuration");
    return;
  }
  const SwipeLayout lay = swipe_layout(pv.L1, a.slot, a.rpw, a.tile_records, a.codes_cap, fb, letter_form(a));
  const int per_cu = std::max(1, std::min(8, 160 * 1024 / std::max(lay.total, 1)));
  // MOC_SWIPE_SLOTS (test hook): a smaller persistent grid, so modest batches reach the tail-tile region
  static const int64_t slots_override = [] {
    const char* v = std::getenv("MOC_SWIPE_SLOTS");
    return v ? std::max<int64_t>(1, std::atoll(v)) : int64_t{0};
  }();
  const int64_t slots = slots_override ? slots_override : static_cast<int64_t>(num_cus) * per_cu;
  ShortArgs b = a;
  // the last `slots` tiles' records go in quarter tiles (MOC_SWIPE_TAIL): the tail of the persistent grid
  // (blocks idling while the last tiles finish) shrinks 4x
  const int64_t n_big = (a.n + a.tile_records - 1) / a.tile_records;
  const int div = tail_div();
  if (div && a.tile_records % (64 * div) == 0 && n_big > 2 * slots) {  // tail tiles: multiples of 64 records
    b.tail_from = n_big - slots;
    b.tail_records = a.tile_records / div;
  }
  const int64_t big_end = b.tail_records ? b.tail_from * b.tile_records : b.n;
  const int64_t n_tiles =
      b.tail_records ? b.tail_from + (b.n - big_end + b.tail_records - 1) / b.tail_records : n_big;
  const int64_t blocks = std::min<int64_t>(n_tiles, slots);
  const dim3 grid(static_cast<unsigned>(std::max<int64_t>(blocks, 1))), block(kBlock);
  const bool ok = launch_swipe_instance(letter_form(a), pv, b, lay, grid, block, num_cus, stream);
  if (!ok) throw Error("launch_swipe: no instance for this configuration");
}

}  // namespace dev
}  // namespace moc
