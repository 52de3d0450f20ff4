"""
    MPIAsyncPools

The MI355X-native `asyncmap!` hot path behind the API of MPIAsyncPools.jl
(severinson/MPIStragglers.jl, `src/MPIAsyncPools.jl`): `MPIAsyncPool(n)`,
`asyncmap!(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm; nwait, epoch, tag)` returning
the aliased `repochs`, and `waitall!`.  The pool's state lives in libmpiasyncpools.so (the
C ABI of include/mpiasyncpools.h); its fields are `unsafe_wrap`ped arrays over that state,
so `repochs` returned by `asyncmap!` is the same vector later calls mutate
(src/MPIAsyncPools.jl:187).  `comm` is

  * a `DeviceComm`: device workers on HIP streams of this process's GPU, replacing
    `MPI.COMM_WORLD` plus the `worker_main` ranks (BASELINE configs[1], one GPU);
  * a `DistComm`: one process per GPU, as `mpiexec -n N julia ...` ranks (configs[2]-[4] on
    8 GPUs): every rank constructs it with the same placement, rank 0 calls `asyncmap!`,
    the others `serve!` their workers (examples/iterative_example.jl:84-88's rank split);
  * or, with MPI.jl loaded (package extension `MPIAsyncPoolsMPIExt`), a real `MPI.Comm`
    whose ranks run arbitrary worker programs (test/kmap1.jl, test/kmap2.jl unchanged).

UNEXECUTED: Julia is not installed in the build image.  This module is written against the
header and kept in sync mechanically by `tests/test_abi_table.py` (its `ccall`s come from the
generated capi.jl, every `mpa_*` it calls exists in the signature table with the right
arity); the Python binding drives the same ABI in every test, and a C client of the ABI
(`tests/c/capi_client.c`) runs it with exact-size device buffers on the GPU.  Its own
behaviour (argument checks, conversions) is parity unpinned.
"""
module MPIAsyncPools

export MPIAsyncPool, waitall!, DeviceComm, DistComm, set_task_lsq!, set_task_lsq_batch!, set_task_kmap!,
       set_delays!, shutdown!, serve!, pause_servers!, payload_path, lsq_descent!, lsqb_descent!, first_plus

const libmpiasyncpools = get(ENV, "MPA_LIB",
                             joinpath(@__DIR__, "..", "..", "..", "mpistragglers.jl_amd", "_build", "libmpiasyncpools.so"))

include("capi.jl")

# status codes -> the reference's exceptions (src/MPIAsyncPools.jl:71-77,157)
const MPA_OK, MPA_ARGUMENT_ERROR, MPA_DIMENSION_MISMATCH, MPA_ERROR = 0, 1, 2, 3
const MPA_NWAIT_INT, MPA_NWAIT_FN, MPA_NWAIT_OTHER = 0, 1, 2
const MPA_TRANSPORT_HIP, MPA_TRANSPORT_HOST = 0, 2
const MPA_TASK_ECHO, MPA_TASK_KMAP1, MPA_TASK_KMAP2 = 1, 2, 3
const MPA_F32, MPA_F64, MPA_BF16 = 0, 1, 2
const LSQB_ITERATES = 64  # iterates per message of the batched variant (include/mpiasyncpools.h)

function check(rc::Integer)
    rc == MPA_OK && return nothing
    msg = unsafe_string(mpa_last_error())
    rc == MPA_ARGUMENT_ERROR && throw(ArgumentError(msg))
    rc == MPA_DIMENSION_MISMATCH && throw(DimensionMismatch(msg))
    error(msg)
end

function __init__()
    v = mpa_abi_version()
    v == MPA_ABI_VERSION || error("libmpiasyncpools ABI version $v, this binding expects $MPA_ABI_VERSION")
end

# Buffers cross the ABI as (pointer, bytes).  Only dense arrays have a data pointer and a
# byte count; `sizeof` of a wrapper type is the wrapper's size, not its data's, so bytes are
# length * element size.  Whether the memory is the GPU's is checked by the library (a
# DeviceComm refuses host memory with an ArgumentError).
function _ptr(a)
    a isa DenseArray || throw(ArgumentError("expected a dense (device) array, got $(typeof(a))"))
    return convert(Ptr{Cvoid}, pointer(a))
end
_nbytes(a) = length(a) * sizeof(eltype(a))

"""
    MPIAsyncPool(ranks; epoch0=0, nwait=length(ranks))    # src/MPIAsyncPools.jl:35-43
    MPIAsyncPool(n)                                       # :46

State owned by the library; `ranks, sepochs, repochs, active, stimestamps, latency` alias it.
"""
mutable struct MPIAsyncPool
    h::Ptr{Cvoid}
    ranks::Vector{Int}
    sepochs::Vector{Int}
    repochs::Vector{Int}
    active::Vector{Bool}
    stimestamps::Vector{Int}
    latency::Vector{Float64}
end

function MPIAsyncPool(ranks::AbstractVector{<:Integer}; epoch0::Integer=0, nwait::Integer=length(ranks))
    r = Vector{Int64}(ranks)
    n = length(r)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(mpa_pool_create(n, r, epoch0, nwait, h))
    wrap(p, T) = unsafe_wrap(Array, convert(Ptr{T}, p), n; own=false)
    pool = MPIAsyncPool(h[], wrap(mpa_pool_ranks(h[]), Int), wrap(mpa_pool_sepochs(h[]), Int),
                        wrap(mpa_pool_repochs(h[]), Int), wrap(mpa_pool_active(h[]), Bool),
                        wrap(mpa_pool_stimestamps(h[]), Int), wrap(mpa_pool_latency(h[]), Float64))
    finalizer(p -> (p.h != C_NULL && mpa_pool_destroy(p.h); p.h = C_NULL), pool)
end
MPIAsyncPool(n::Integer; kwargs...) = MPIAsyncPool(collect(1:n); kwargs...)

# pool.epoch / pool.nwait are scalars of the library's state (src/MPIAsyncPools.jl:33-34)
function Base.getproperty(p::MPIAsyncPool, s::Symbol)
    s === :epoch && return Int(unsafe_load(mpa_pool_epoch(getfield(p, :h))))
    s === :nwait && return Int(unsafe_load(mpa_pool_nwait(getfield(p, :h))))
    return getfield(p, s)
end
function Base.setproperty!(p::MPIAsyncPool, s::Symbol, v)
    s === :epoch && return unsafe_store!(mpa_pool_epoch(getfield(p, :h)), Int64(v))
    s === :nwait && return unsafe_store!(mpa_pool_nwait(getfield(p, :h)), Int64(v))
    return setfield!(p, s, v)
end
Base.length(p::MPIAsyncPool) = length(getfield(p, :ranks))

"""A communicator handle of the library: the `comm` argument of `asyncmap!`."""
abstract type AbstractComm end

"""
    DeviceComm(nworkers)

The `comm::MPI.Comm` of the reference together with its worker ranks: `nworkers` device
workers (ranks 1..nworkers) on this process's current GPU, each running a registered task on
its own HIP stream.  (Workers on other GPUs are served by their own processes: `DistComm`.)
"""
mutable struct DeviceComm <: AbstractComm
    h::Ptr{Cvoid}
    keep::Dict{Int,Any}   # device arrays of registered tasks stay alive with the comm
end
function DeviceComm(nworkers::Integer)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(mpa_comm_create(MPA_TRANSPORT_HIP, nworkers, C_NULL, h))
    c = DeviceComm(h[], Dict{Int,Any}())
    finalizer(c -> (c.h != C_NULL && mpa_comm_destroy(c.h); c.h = C_NULL), c)
end
DeviceComm(h::Ptr{Cvoid}) = DeviceComm(h, Dict{Int,Any}())

"""
    DistComm(nworkers, placement, rank, shm_name, max_msg_bytes; transport=:hip)

One process per GPU (DESIGN.md §5), the shape `mpiexec -n N julia script.jl` gives the
reference (examples/iterative_example.jl:84-88): `placement[w]` is the process rank serving
worker `w` (0 = the coordinator's own process), every rank constructs the comm with the same
arguments, rank 0 first (it creates the shared-memory mailboxes `shm_name`, messages of at
most `max_msg_bytes` each way; MPI.Bcast the name, then construct on the other ranks).  Rank
0 calls `asyncmap!` / `waitall!`; every other rank registers its workers' tasks and calls
`serve!`, which returns when rank 0 calls `pause_servers!` or `shutdown!`.  `transport=:host`
runs the same protocol with host-executed test workers and no GPU.
"""
mutable struct DistComm <: AbstractComm
    h::Ptr{Cvoid}
    keep::Dict{Int,Any}
    rank::Int
end
function DistComm(nworkers::Integer, placement::AbstractVector{<:Integer}, rank::Integer, shm_name::AbstractString,
                  max_msg_bytes::Integer; transport::Symbol=:hip)
    length(placement) == nworkers || throw(DimensionMismatch("placement has $(length(placement)) entries, $nworkers workers"))
    code = transport === :hip ? MPA_TRANSPORT_HIP : transport === :host ? MPA_TRANSPORT_HOST :
           throw(ArgumentError("transport must be :hip or :host"))
    pl = Vector{Cint}(placement)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve pl check(mpa_comm_create_dist(code, nworkers, pointer(pl), rank, shm_name, max_msg_bytes, h))
    c = DistComm(h[], Dict{Int,Any}(), Int(rank))
    finalizer(c -> (c.h != C_NULL && mpa_comm_destroy(c.h); c.h = C_NULL), c)
end

"""serve!(comm::DistComm): worker processes run the tasks posted to their workers (the
reference's `worker_main` loop, examples/iterative_example.jl:55-82) until rank 0 pauses or
shuts the comm down."""
serve!(c::DistComm) = check(mpa_comm_serve(c.h))
"""pause_servers!(comm::DistComm): rank 0 makes every running `serve!` return (e.g. before
a barrier between phases)."""
pause_servers!(c::DistComm) = check(mpa_comm_pause_servers(c.h))
"""payload_path(comm::DistComm, rank): `:device` (xGMI, HIP IPC), `:host` (shared-memory
mailbox) or `nothing` (undecided / served by rank 0) for worker `rank`."""
function payload_path(c::DistComm, rank::Integer)
    p = mpa_comm_payload_path(c.h, rank)
    return p == 2 ? :device : p == 1 ? :host : nothing
end

"""
    set_task_lsq!(comm, rank, At, b)

Worker `rank` computes g = A^T (A x - b).  The kernel reads A row-major, which is a
column-major Julia matrix `At` of size cols x rows (lda = size(At, 1)); `b` has rows elements.
"""
function set_task_lsq!(c::AbstractComm, rank::Integer, At::AbstractMatrix{T}, b::AbstractVector{T}) where {T<:Union{Float32,Float64}}
    size(At, 2) == length(b) || throw(DimensionMismatch("A has $(size(At, 2)) rows, b has $(length(b)) elements"))
    check(mpa_comm_set_task_lsq(c.h, rank, T === Float64 ? MPA_F64 : MPA_F32, size(At, 2), size(At, 1), _ptr(At),
                                size(At, 1), _ptr(b)))
    c.keep[Int(rank)] = (At, b)
    return nothing
end

"""
    set_task_lsq_batch!(comm, rank, At, Bt)

Worker `rank` computes the batched variant G = A^T (A X - B) for 64 iterates (BASELINE
configs[4]): bf16 A and B, fp32 G.  `At` is cols x rows (a column-major Julia matrix = A
row-major, lda = size(At, 1)), `Bt` is 64 x rows (= B row-major), both of 2-byte elements
holding bf16 bits (`BFloat16` or `UInt16`).  The message X is cols x 64 bf16 and the reply G
cols x 64 Float32, both row-major (64 x cols column-major Julia matrices).
"""
function set_task_lsq_batch!(c::AbstractComm, rank::Integer, At::AbstractMatrix, Bt::AbstractMatrix)
    sizeof(eltype(At)) == 2 && sizeof(eltype(Bt)) == 2 || throw(ArgumentError("A and B hold bf16 (2-byte) elements"))
    size(Bt, 1) == LSQB_ITERATES || throw(DimensionMismatch("B must be $LSQB_ITERATES x rows, is $(size(Bt))"))
    size(At, 2) == size(Bt, 2) || throw(DimensionMismatch("A has $(size(At, 2)) rows, B has $(size(Bt, 2))"))
    check(mpa_comm_set_task_lsq_batch(c.h, rank, size(At, 2), size(At, 1), LSQB_ITERATES, _ptr(At), size(At, 1), _ptr(Bt)))
    c.keep[Int(rank)] = (At, Bt)
    return nothing
end

"""set_task_kmap!(comm, rank, :kmap1 | :kmap2 | :echo): the reference's test worker programs
(test/kmap1.jl:23-33, test/kmap2.jl:76-99) as device tasks."""
set_task_kmap!(c::AbstractComm, rank::Integer, task::Symbol) =
    check(mpa_comm_set_task_kmap(c.h, rank, task === :kmap1 ? MPA_TASK_KMAP1 : task === :kmap2 ? MPA_TASK_KMAP2 :
                                            task === :echo ? MPA_TASK_ECHO : throw(ArgumentError("unknown task $task"))))

"""set_delays!(comm, rank, delays_ns): task t of the worker sleeps delays_ns[(t-1) % end + 1]
before it computes (the reference worker's `sleep`, test/kmap2.jl:95)."""
function set_delays!(c::AbstractComm, rank::Integer, delays_ns::AbstractVector{<:Integer})
    d = Vector{Int64}(delays_ns)
    GC.@preserve d check(mpa_comm_set_delays(c.h, rank, isempty(d) ? C_NULL : pointer(d), length(d)))
end

"""shutdown!(comm): the control-tag shutdown (examples/iterative_example.jl:49-52): drain the
outstanding tasks, then refuse further posts."""
shutdown!(c::AbstractComm) = check(mpa_comm_shutdown(c.h))

# nwait::Function (src/MPIAsyncPools.jl:153): the library calls back on the caller's thread
# with the pool's repochs; the function travels in the callback's context pointer (per call,
# per pool: no global state)
function _nwait_trampoline(ctx::Ptr{Cvoid}, epoch::Int64, repochs::Ptr{Int64}, n::Int64)::Cint
    try
        f = unsafe_pointer_to_objref(ctx)::Base.RefValue{Any}
        return f[](epoch, unsafe_wrap(Array, repochs, n; own=false))::Bool ? Cint(1) : Cint(0)
    catch
        return Cint(-1)
    end
end

"""first_plus(k): nwait that holds once worker 1 and at least k of the others are fresh (the
predicate of test/kmap2.jl:65 widened to k-of-n; evaluated natively, mpa_nwait_first_plus)."""
struct FirstPlus
    k::Int64
end
first_plus(k::Integer) = FirstPlus(k)

"""
    asyncmap!(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm; nwait, epoch, tag)

src/MPIAsyncPools.jl:68-188 over the library's transport.  Returns `pool.repochs` (aliased).
"""
function Base.asyncmap!(pool::MPIAsyncPool, sendbuf, recvbuf, isendbuf, irecvbuf, comm::AbstractComm;
                        nwait::Union{<:Integer,Function,FirstPlus}=pool.nwait, epoch::Integer=pool.epoch + 1,
                        tag::Integer=0)
    isbitstype(eltype(sendbuf)) || throw(ArgumentError("The eltype of sendbuf must be isbits, but is $(eltype(sendbuf))"))
    isbitstype(eltype(recvbuf)) || throw(ArgumentError("The eltype of sendbuf must be isbits, but is $(eltype(recvbuf))"))
    ctxref = Ref{Any}(nwait)
    kctx = Ref{Int64}(nwait isa FirstPlus ? nwait.k : 0)
    if nwait isa Integer
        kind, k, fn, ctx = MPA_NWAIT_INT, Int64(nwait), C_NULL, C_NULL
    elseif nwait isa FirstPlus
        kind, k = MPA_NWAIT_FN, Int64(0)
        fn = cglobal((:mpa_nwait_first_plus, libmpiasyncpools))
        ctx = Base.unsafe_convert(Ptr{Int64}, kctx)
    else
        kind, k = MPA_NWAIT_FN, Int64(0)
        fn = @cfunction(_nwait_trampoline, Cint, (Ptr{Cvoid}, Int64, Ptr{Int64}, Int64))
        ctx = pointer_from_objref(ctxref)
    end
    GC.@preserve ctxref kctx sendbuf recvbuf isendbuf irecvbuf begin
        check(mpa_asyncmap(pool.h, _ptr(sendbuf), _nbytes(sendbuf), _ptr(recvbuf), _nbytes(recvbuf), length(recvbuf),
                           _ptr(isendbuf), _nbytes(isendbuf), _ptr(irecvbuf), _nbytes(irecvbuf), comm.h,
                           kind, k, fn, convert(Ptr{Cvoid}, ctx), string(typeof(nwait)), epoch, tag,
                           Ptr{Ptr{Int64}}(C_NULL)))
    end
    return pool.repochs                      # the aliased vector, :187
end

"""waitall!(pool, recvbuf, irecvbuf)  (src/MPIAsyncPools.jl:195-224)"""
function waitall!(pool::MPIAsyncPool, recvbuf, irecvbuf)
    isbitstype(eltype(recvbuf)) || throw(ArgumentError("The eltype of sendbuf must be isbits, but is $(eltype(recvbuf))"))
    GC.@preserve recvbuf irecvbuf begin
        check(mpa_waitall(pool.h, _ptr(recvbuf), _nbytes(recvbuf), length(recvbuf), _ptr(irecvbuf), _nbytes(irecvbuf),
                          Ptr{Ptr{Int64}}(C_NULL)))
    end
    return pool.repochs
end

"""
    lsq_descent!(pool, comm, x, recvbuf, isendbuf, irecvbuf; nwait, eta, epochs, stale_weight=0.0)

The coordinator loop of examples/iterative_example.jl:37-47 with the least-squares workload,
in native code: `epochs` iterations of asyncmap! followed by the device iterate update
x -= eta * n/sum(w) * sum_i w_i g_i (w_i = 1 fresh, stale_weight for an older result, 0 for a
worker never heard from).
"""
function lsq_descent!(pool::MPIAsyncPool, comm::AbstractComm, x::AbstractVector{T}, recvbuf, isendbuf, irecvbuf;
                      nwait::Union{Integer,FirstPlus}, eta::Real, epochs::Integer,
                      stale_weight::Real=0.0) where {T<:Union{Float32,Float64}}
    kctx = Ref{Int64}(nwait isa FirstPlus ? nwait.k : 0)
    GC.@preserve kctx x recvbuf isendbuf irecvbuf begin
        kind, k, fn, ctx = _native_nwait(nwait, kctx)
        check(mpa_lsq_descent(pool.h, comm.h, T === Float64 ? MPA_F64 : MPA_F32, _ptr(x), length(x),
                              _ptr(recvbuf), _nbytes(recvbuf), _ptr(isendbuf), _nbytes(isendbuf),
                              _ptr(irecvbuf), _nbytes(irecvbuf), kind, k, fn, ctx, eta, stale_weight, epochs))
    end
    return pool.repochs
end

# nwait of the native loops: an Integer, or first_plus(k) evaluated by the library
_native_nwait(nwait, kctx) = nwait isa FirstPlus ?
    (MPA_NWAIT_FN, Int64(0), cglobal((:mpa_nwait_first_plus, libmpiasyncpools)),
     convert(Ptr{Cvoid}, Base.unsafe_convert(Ptr{Int64}, kctx))) :
    (MPA_NWAIT_INT, Int64(nwait), C_NULL, C_NULL)

"""
    lsqb_descent!(pool, comm, x32, xb16, recvbuf, isendbuf, irecvbuf; nwait, eta, epochs, stale_weight=0.0)

The batched variant's coordinator loop (BASELINE configs[4]) in native code: the message is
`xb16` (cols x 64 bf16, the bf16 image of the Float32 iterate `x32`), the replies are
Float32 G_i; each epoch x32 -= eta * n/sum(w) * sum_i w_i G_i and xb16 = bf16(x32), on the
device.
"""
function lsqb_descent!(pool::MPIAsyncPool, comm::AbstractComm, x32::AbstractArray{Float32}, xb16::AbstractArray,
                       recvbuf, isendbuf, irecvbuf; nwait::Union{Integer,FirstPlus}, eta::Real, epochs::Integer,
                       stale_weight::Real=0.0)
    sizeof(eltype(xb16)) == 2 && length(xb16) == length(x32) ||
        throw(DimensionMismatch("xb16 must hold the bf16 image of x32 (2-byte elements, same length)"))
    kctx = Ref{Int64}(nwait isa FirstPlus ? nwait.k : 0)
    GC.@preserve kctx x32 xb16 recvbuf isendbuf irecvbuf begin
        kind, k, fn, ctx = _native_nwait(nwait, kctx)
        check(mpa_lsqb_descent(pool.h, comm.h, _ptr(x32), _ptr(xb16), length(x32),
                               _ptr(recvbuf), _nbytes(recvbuf), _ptr(isendbuf), _nbytes(isendbuf),
                               _ptr(irecvbuf), _nbytes(irecvbuf), kind, k, fn, ctx, eta, stale_weight, epochs))
    end
    return pool.repochs
end

end # module
