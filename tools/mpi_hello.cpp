// The floor of `mpiexec -np N ./final` on a tiny input: a bare MPI program (init, rank, finalize) under the
// same mpiexec (tools/final_walltime_r3.sh). Build: see that script.
#include <mpi.h>

#include <cstdio>

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  if (rank == 0) std::printf("hello\n");
  MPI_Finalize();
  return 0;
}
