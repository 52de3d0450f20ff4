/*
 * mpiasyncpools_mpi.h — the MPI transport of the `asyncmap!` C ABI
 * (libmpiasyncpools_mpi.so, built only where an MPI implementation is present; it links
 * libmpi and libmpiasyncpools.so).
 *
 * Reference interface replaced: the `comm::MPI.Comm` argument of
 *     Base.asyncmap!(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm; ...)
 * (src/MPIAsyncPools.jl:68) when its ranks run ARBITRARY worker programs, as in
 * examples/iterative_example.jl:55-82, test/kmap1.jl:23-33 and test/kmap2.jl:76-99.
 * The pool then drives MPI exactly as the reference does (Isend + Irecv! :137-138,
 * Test! :99, Waitany! :161, Waitall! :212, Wait! on the send :113).  Buffers are host
 * pointers.  The returned handle is used with mpa_asyncmap / mpa_waitall / mpa_comm_destroy
 * of mpiasyncpools.h like any other communicator.
 */
#ifndef MPIASYNCPOOLS_MPI_H
#define MPIASYNCPOOLS_MPI_H

#include <stdint.h>

#include "mpiasyncpools.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mpi_comm_f: the communicator's Fortran handle (MPI_Comm_c2f(comm); in Julia,
 * MPI.jl's `comm.val` for MPICH-ABI libraries).  Workers are ranks 1..size-1 of it; the
 * caller (the coordinator) must have initialised MPI.  Status codes as mpiasyncpools.h. */
int mpa_comm_create_mpi(int64_t mpi_comm_f, mpa_comm** out);

#ifdef __cplusplus
}
#endif

#endif
