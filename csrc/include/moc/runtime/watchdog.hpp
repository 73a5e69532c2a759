// Deadline on every blocking communication wait.
//
// Reference: a failing rank exit(1)s without MPI_Abort (/root/reference/cudaFunctions.cu:15-33) and its
// peers block forever in the next rooted collective (main.c:174,195-197). Here every wait of the
// distributed layer — MPI requests (moc/comm.hpp), the MPI-emulated device comm, and the RCCL comm lane's
// stream/event queries with ncclCommGetAsyncError (the GPU plugin) — polls against one job-wide deadline
// (--comm-timeout / MOC_COMM_TIMEOUT seconds, 0 = wait forever). When it passes, the wait throws
// CommTimeout naming the rank, the job's phase, the operation and what is still outstanding; the caller's
// fail-fast path turns that into MPI_Abort, so a stuck peer ends the job with a diagnosis instead of a
// silent hang.
#pragma once

#include <cstdint>
#include <functional>
#include <string>

#include "moc/common.hpp"

namespace moc {

struct CommTimeout : Error {
  using Error::Error;
};

namespace watchdog {

constexpr double kDefaultTimeoutS = 300.0;

// <= 0 disables the deadline. Process-wide (each shared object that links the runtime keeps its own copy:
// the GPU plugin is given the job's value through GpuRankOptions).
void set_timeout_s(double s);
double timeout_s();
// The job's current phase (PhaseTimer::begin sets it), named by timeouts and fatal errors.
void set_phase(const char* phase);
std::string phase();
void set_rank(int rank);
int rank();

// How a wait polls. Busy: `done()` back to back, as MPI_Waitall does — MPICH moves a large message's data
// inside its progress calls, so a sleeping poller would slow the transfer itself. Backoff: spin for the
// first ~2 ms, then sleep up to 1 ms between polls — for work the device (or RCCL's proxy thread) does
// without this thread.
enum class Poll { Busy, Backoff };

struct WaitSpec {
  const char* what = "";                      // the operation, for the message
  std::function<std::string()> outstanding;   // what is still pending (called once, at expiry)
  std::function<void()> check;                // every ~1 ms; may throw (RCCL's asynchronous error)
  std::function<void()> expire;               // at expiry, before the throw (e.g. ncclCommAbort)
  Poll poll = Poll::Busy;
};

// Polls `done()` until it returns true; past the deadline runs spec.expire and throws CommTimeout.
void wait(const std::function<bool()>& done, const WaitSpec& spec);

// "1.5 MiB"-style byte counts for the messages.
std::string human_bytes(int64_t bytes);

}  // namespace watchdog
}  // namespace moc
