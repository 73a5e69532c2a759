/* Flat C ABI of libmoc.so — consumed by the Python package through ctypes (no pybind/torch build
 * dependency, so the same shared object serves the CLI, the tests and the torch-facing ops).
 * Every function returns 0 on success or -1 on error (message: moc_last_error()). */
#ifndef MOC_CAPI_H_
#define MOC_CAPI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct moc_result {
  int32_t score, n, k;
} moc_result;

const char* moc_last_error(void);
int moc_abi_version(void);
int moc_set_log_level(const char* level);

/* ---- problem / io ---- */
void* moc_parse(const char* data, size_t len, int strict_limits);
void moc_problem_free(void* p);
int moc_problem_info(void* p, int32_t* weights4, int64_t* L1, int64_t* n, int64_t* total_chars);
const uint8_t* moc_problem_seq1(void* p);
const uint8_t* moc_problem_codes(void* p);
const int64_t* moc_problem_offsets(void* p);
/* Formats rows into buf (cap bytes); returns bytes written or -1 (needs ~96 B per row). */
int64_t moc_format_results(const moc_result* r, int64_t n, int64_t first_index, char* buf, int64_t cap);

/* ---- 5-bit packed letter codes (moc/problem.hpp) ---- */
int64_t moc_packed5_bytes(int64_t n_chars);
int moc_pack5(const uint8_t* codes, int64_t n, uint8_t* out);
int moc_unpack5(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out);
// 33-bit fields: 7 letters per field, 56 letters per 33 bytes (moc::pack33, 4.714 bits per letter)
int64_t moc_packed33_bytes(int64_t n_chars);
int moc_pack33(const uint8_t* codes, int64_t n, uint8_t* out);
int moc_unpack33(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out);
// narrow record lengths from CSR offsets (moc::pack_lengths): bits 3 / 4 / 8, or 6 = base-6 octets
int moc_pack_lengths(const int64_t* offsets, int64_t n, int bits, int64_t base, uint8_t* out);

/* ---- score table ---- */
int moc_score_table(const int32_t* weights4, int32_t* lut1024, uint8_t* cls1024);

/* ---- exactness bounds of the kernels' narrow-integer forms (moc/kernel_bounds.hpp); no GPU needed ----
 * out6: [0] swipe key form (moc::bounds::kFormSwipeKBits / kFormSwipeRK, 0 = the swipe kernel's integer
 * bounds refuse the batch), [1] 1 if the short kernel's packed int16 form is exact, [2] the int32 hot-key
 * shift of the short / tile kernels (0 = 64-bit keys), [3] 1 if the tile16 profile holds the table, [4] the
 * index bits of tile16's 32-bit selection keys (0 = 64-bit keys), [5] 1 if the int16 tile16 profile holds the
 * table. */
int moc_kernel_bounds(const int32_t* weights4, int64_t L1, int64_t min_l2, int64_t max_l2, int32_t* out6);
/* "src=<source hash> defs=<-D flags of the kernel objects>" (empty defs: the product build) */
const char* moc_build_info(void);

/* ---- CPU engine (OpenMP) ---- */
int moc_cpu_solve(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                  const int64_t* offsets, int64_t n, int semantics, int threads, moc_result* out);
int moc_brute_force(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                    const int64_t* offsets, int64_t n, int semantics, moc_result* out);

/* ---- context-parallel partial searches (packed 64-bit keys; 0 = no candidate) ---- */
int moc_cpu_solve_keys(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                       const int64_t* offsets, int64_t n, int semantics, int part, int parts, int threads,
                       uint64_t* keys);
/* MAX-combined pass-1 keys -> results: k resolved on each record's winning diagonal (needs the batch). */
int moc_resolve_keys(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                     const int64_t* offsets, int64_t n, const uint64_t* keys, moc_result* out);

/* ---- partition ---- */
int moc_partition(const int64_t* lengths, int64_t n, int64_t L1, int parts, double cell_w, double byte_w,
                  double record_w, int64_t* bounds_out /* parts+1 */);

/* ---- HIP engine ---- */
int moc_device_count(void);
/* Page-locks [p, p+bytes) for direct DMA (hipHostRegister on the enclosing page range). */
int moc_host_register(void* p, size_t bytes);
// Page-locked host allocation known to the streaming paths (nullptr on failure; moc_last_error).
void* moc_host_alloc(size_t bytes);
int moc_host_free(void* p);
/* Binds CPUs + future host allocations of this process to the device's NUMA node; returns node or -1. */
int moc_bind_numa(int device);
int moc_device_numa_node(int device);
/* Runs the DPP/shuffle self-test kernel; fills 192 ints (layout: align_kernels.hip dpp_probe_kernel). */
int moc_dpp_probe(int32_t* out192);
/* i8 MFMA layout self-test: c = a * b for row-major 32x32 int8 a, b (tile_mfma_kernels.hip). */
int moc_mfma_i8_probe(const int8_t* a32x32, const int8_t* b32x32, int32_t* c32x32);
/* Transfer calibration: GB/s for kind 0 H2D, 1 D2H, 2 both, 3 zero-copy read, 4 zero-copy write, 5 D2D. */
double moc_transfer_probe(int kind, size_t bytes, int iters);
/* out6: type, hostPointer, devicePointer, hipHostGetDevicePointer, hipMemGetAddressRange base, size */
int moc_pointer_info(const void* p, size_t bytes, uint64_t* out6);
/* 1 when every byte of [p, p+bytes) is page-locked through this library's registry */
int moc_pinned_covers(const void* p, size_t bytes);
int moc_host_unregister(void* p);
int moc_device_info_json(int device, char* buf, int64_t cap);
void* moc_engine_create(int device, int64_t chunk_records, int64_t chunk_bytes, int allow_direct);
void moc_engine_destroy(void* e);
int moc_engine_set_problem(void* e, const int32_t* weights4, const uint8_t* seq1, int64_t L1, int semantics);
int moc_engine_solve(void* e, const uint8_t* codes, const int64_t* offsets, int64_t n, moc_result* out);
/* fmt: 0 = R12 (moc_result), 1 = R8 {i32,u16,u16}, 2 = R4 {i16,u8,u8}, 3 = R2 (u16 mixed-radix code,
 * moc_engine_r2_params); lengths (len_bits 8, or 4 = two per byte, value + len_base) / min_l2 / max_l2
 * optional (NULL / -1). Pinned host buffers + short records -> zero-copy streaming kernel. */
int moc_engine_solve_ex(void* e, const uint8_t* codes, const int64_t* offsets, const uint8_t* lengths, int len_bits,
                        int len_base, int64_t n, void* out, int fmt, int64_t min_l2, int64_t max_l2,
                        int packed);  // packed: 0 byte letters, 1 5-bit packed, 3 P33 fields
int moc_engine_auto_format(void* e, int64_t max_l2, int64_t min_l2);
/* R2 parameters {smin, kw, j} for records with lengths in [min_l2, max_l2] */
int moc_engine_r2_params(void* e, int64_t min_l2, int64_t max_l2, int32_t* out3);
int moc_engine_pin(void* e, const void* p, size_t bytes);

// Device-resident batch in the wire formats (every pointer device memory of the engine's GPU; packed 3 =
// P33 letters, 0 = bytes; dense offsets; narrow lengths as in moc_engine_solve_ex): the swipe kernel reads
// them in place (the rccl transport's path, csrc/src/device_batch.cpp). Synchronous; stats give the
// kernel time.
int moc_engine_solve_wire_device(void* e, const uint8_t* d_letters, const int64_t* d_offsets, const uint8_t* d_lengths,
                                 int len_bits, int len_base, int64_t n, void* d_out, int fmt, int64_t min_l2,
                                 int64_t max_l2, int packed);
// device time (ms) of the last moc_engine_solve_device's kernels; waits for them
int moc_engine_device_kernel_ms(void* e, double* ms);
int moc_engine_solve_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                            int64_t n, moc_result* d_out, void* stream);
int moc_engine_search_keys(void* e, const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                           uint64_t* keys);
int moc_engine_search_keys_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                  int64_t n, int part, int parts, uint64_t* d_keys, void* stream);
int moc_engine_finalize_keys_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                    int64_t n, const uint64_t* d_keys, void* d_out,
                                    int fmt, void* stream);
/* stats: kernel_ms, total_ms, h2d_bytes, d2h_bytes, chunks, cells, records, direct, format, kernels,
 * r2 smin, r2 kw, r2 j, forms (moc::bounds::FormBits of the last solve) */
int moc_engine_stats(void* e, double* out14);

#ifdef __cplusplus
}
#endif

#endif
