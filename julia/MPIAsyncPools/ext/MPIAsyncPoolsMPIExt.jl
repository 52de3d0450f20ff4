"""
The `asyncmap!` / `waitall!` methods for a real `MPI.Comm` (loaded with MPI.jl): the pool of
libmpiasyncpools.so driven over libmpiasyncpools_mpi.so, whose transport is the reference's
own MPI verbs (Isend + Irecv!, Test!, Waitany!, Waitall!; src/MPIAsyncPools.jl:99,113,137-138,
161,212), so test/kmap1.jl and test/kmap2.jl run unchanged, worker ranks included.  Buffers
are host arrays.  (UNEXECUTED here, see the module docstring; the C equivalent of this root
side, tests/mpi/pool_mpi_kmap.c, runs the golden kmap2 scenarios over MPICH in the tests.)
"""
module MPIAsyncPoolsMPIExt

using MPI
using MPIAsyncPools
using MPIAsyncPools: AbstractComm, MPIAsyncPool, check, mpa_comm_destroy

const libmpi_t = get(ENV, "MPA_MPI_LIB",
                     joinpath(@__DIR__, "..", "..", "..", "mpistragglers.jl_amd", "_build", "libmpiasyncpools_mpi.so"))

"""A communicator handle of the MPI transport (mpa_comm_create_mpi, include/mpiasyncpools_mpi.h)."""
mutable struct MPITransportComm <: AbstractComm
    h::Ptr{Cvoid}
    keep::Dict{Int,Any}
end

const HANDLES = IdDict{MPI.Comm,MPITransportComm}()  # one transport per communicator, for the pool's lifetime

function transport(comm::MPI.Comm)
    get!(HANDLES, comm) do
        h = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:mpa_comm_create_mpi, libmpi_t), Cint, (Int64, Ptr{Ptr{Cvoid}}), fortran_handle(comm), h))
        c = MPITransportComm(h[], Dict{Int,Any}())
        finalizer(c -> (c.h != C_NULL && mpa_comm_destroy(c.h); c.h = C_NULL), c)
    end
end

# the Fortran handle of a communicator (mpa_comm_create_mpi takes MPI_Comm_c2f's value, which
# does not depend on the C handle type of the MPI library MPI.jl loaded)
fortran_handle(comm::MPI.Comm) = Int64(ccall((:MPI_Comm_c2f, MPI.libmpi), Cint, (MPI.MPI_Comm,), comm))

Base.asyncmap!(pool::MPIAsyncPool, sendbuf, recvbuf, isendbuf, irecvbuf, comm::MPI.Comm; kwargs...) =
    asyncmap!(pool, sendbuf, recvbuf, isendbuf, irecvbuf, transport(comm); kwargs...)

end # module
