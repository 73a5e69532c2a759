// HIP error checking — native replacement for the vendored CUDA-Samples checkCudaErrors /
// getLastCudaError (inc/helper_cuda.h:566-614) and for the reference's checkStatus/checkStatusInt
// (cudaFunctions.cu:15-33), which called host free() on device/constant pointers and exit(1)
// without MPI_Abort (bug B11). Errors here throw moc::Error("<file>:<line> <call>: <hip message>");
// the CLI turns any exception into MPI_Abort so peer ranks never hang in a collective.
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>

#include "moc/common.hpp"

namespace moc {

[[noreturn]] inline void throw_hip(hipError_t e, const char* what, const char* file, int line) {
  (void)hipGetLastError();  // the failure is reported here: do not leave it to the next API call on this thread
  throw Error(std::string(file) + ":" + std::to_string(line) + " " + what + ": " + hipGetErrorName(e) + " (" +
              hipGetErrorString(e) + ")");
}

}  // namespace moc

#define MOC_HIP_CHECK(call)                                                  \
  do {                                                                       \
    hipError_t moc_err_ = (call);                                            \
    if (moc_err_ != hipSuccess) ::moc::throw_hip(moc_err_, #call, __FILE__, __LINE__); \
  } while (0)
