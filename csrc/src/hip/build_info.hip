// Build identity of the kernel objects in this library: the source hash the Makefile computed and the
// extra -D flags the kernels were compiled with. Compiled with every kernel file, so a `make variant` or
// `make debug-kernels` library reports its defines; the product build reports none, and the Python
// loader refuses a library whose kernels carry defines unless MOC_ALLOW_VARIANT_LIB=1
// (mpi_openmp_cuda_amd/_lib.py; tests/test_cli.py checks the in-tree library).
#include <hip/hip_runtime.h>

#ifndef MOC_SRC_HASH
#define MOC_SRC_HASH "unknown"
#endif
#ifndef MOC_KERNEL_DEFS
#ifdef MOC_DEBUG_KERNELS
#define MOC_KERNEL_DEFS "-DMOC_DEBUG_KERNELS"
#else
#define MOC_KERNEL_DEFS ""
#endif
#endif

extern "C" const char* moc_build_info(void) { return "src=" MOC_SRC_HASH " defs=" MOC_KERNEL_DEFS; }
