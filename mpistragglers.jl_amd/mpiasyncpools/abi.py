"""The signature table of the C ABI (include/mpiasyncpools.h), in one place.

Both bindings are generated from it: the ctypes argtypes of `_capi.py` (the tested Python
binding) and the low-level `ccall` wrappers of the Julia module
(`julia/MPIAsyncPools/src/capi.jl`, written by `julia/gen_capi.py`).
`tests/test_abi_table.py` checks that the header declares exactly these prototypes and that
the committed Julia file is what the generator writes, so header, Julia and Python cannot
drift apart.
"""
import re

ABI_VERSION = 3

# one C prototype per entry point, exactly as include/mpiasyncpools.h declares it
PROTOTYPES = """
int mpa_nwait_first_plus(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n);
int mpa_abi_version(void);
const char* mpa_last_error(void);
const char* mpa_build_info(void);
int mpa_tune(const char* key, int64_t value);
int mpa_pool_create(int64_t n, const int64_t* ranks, int64_t epoch0, int64_t nwait, mpa_pool** out);
void mpa_pool_destroy(mpa_pool* pool);
int64_t mpa_pool_size(const mpa_pool* pool);
int64_t* mpa_pool_ranks(mpa_pool* pool);
int64_t* mpa_pool_sepochs(mpa_pool* pool);
int64_t* mpa_pool_repochs(mpa_pool* pool);
uint8_t* mpa_pool_active(mpa_pool* pool);
int64_t* mpa_pool_stimestamps(mpa_pool* pool);
double* mpa_pool_latency(mpa_pool* pool);
int64_t* mpa_pool_nwait(mpa_pool* pool);
int64_t* mpa_pool_epoch(mpa_pool* pool);
int mpa_asyncmap(mpa_pool* pool, const void* sendbuf, size_t sendbuf_bytes, void* recvbuf, size_t recvbuf_bytes, size_t recvbuf_length, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf, size_t irecvbuf_bytes, mpa_comm* comm, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx, const char* nwait_typename, int64_t epoch, int64_t tag, int64_t** repochs_out);
int mpa_waitall(mpa_pool* pool, void* recvbuf, size_t recvbuf_bytes, size_t recvbuf_length, void* irecvbuf, size_t irecvbuf_bytes, int64_t** repochs_out);
int mpa_comm_create(int transport, int64_t nworkers, const int* devices, mpa_comm** out);
void mpa_comm_destroy(mpa_comm* comm);
int64_t mpa_comm_size(const mpa_comm* comm);
int mpa_comm_set_stream(mpa_comm* comm, void* stream);
int mpa_comm_set_task_kmap(mpa_comm* comm, int64_t rank, int task);
int mpa_comm_set_task_lsq(mpa_comm* comm, int64_t rank, int dtype, int64_t rows, int64_t cols, const void* A, int64_t lda, const void* b);
int mpa_comm_set_task_lsq_batch(mpa_comm* comm, int64_t rank, int64_t rows, int64_t cols, int64_t k, const void* A, int64_t lda, const void* B);
int mpa_comm_set_delays(mpa_comm* comm, int64_t rank, const int64_t* delays_ns, int64_t count);
int64_t mpa_comm_tasks_done(mpa_comm* comm, int64_t rank);
int mpa_comm_shutdown(mpa_comm* comm);
int mpa_comm_set_gate(mpa_comm* comm, int64_t nsteps, const int* kinds, const int64_t* offsets, const int64_t* ranks);
int64_t mpa_comm_counter(mpa_comm* comm, const char* name);
int mpa_comm_create_dist(int transport, int64_t nworkers, const int* placement, int my_rank, const char* shm_name, size_t max_msg_bytes, mpa_comm** out);
int mpa_comm_serve(mpa_comm* comm);
int mpa_comm_pause_servers(mpa_comm* comm);
int mpa_comm_payload_path(mpa_comm* comm, int64_t rank);
int mpa_comm_set_timing(mpa_comm* comm, int enable);
int mpa_comm_timing(mpa_comm* comm, double out[4]);
int mpa_comm_exchange_timing(mpa_comm* comm, double out[3]);
int mpa_comm_set_trace(mpa_comm* comm, int64_t capacity);
int mpa_comm_trace(mpa_comm* comm, int64_t* out, int64_t capacity, int64_t* count);
int mpa_comm_sim_set_compute(mpa_comm* comm, int64_t compute_ns);
int mpa_comm_sim_advance(mpa_comm* comm, int64_t dt_ns);
int64_t mpa_comm_sim_now(const mpa_comm* comm);
int mpa_aggregate(mpa_comm* comm, int dtype, const void* recvbuf, int64_t nchunks, int64_t chunk_elems, const double* weights, void* out);
int mpa_lsq_update(mpa_comm* comm, int dtype, void* x, const void* recvbuf, int64_t nchunks, int64_t cols, const double* weights, double eta);
int mpa_lsq_descent(mpa_pool* pool, mpa_comm* comm, int dtype, void* x, int64_t cols, void* recvbuf, size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf, size_t irecvbuf_bytes, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx, double eta, double stale_weight, int64_t epochs);
int mpa_lsqb_update(mpa_comm* comm, void* x32, void* xb16, const void* recvbuf, int64_t nchunks, int64_t elems, const double* weights, double eta);
int mpa_lsqb_descent(mpa_pool* pool, mpa_comm* comm, void* x32, void* xb16, int64_t elems, void* recvbuf, size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf, size_t irecvbuf_bytes, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx, double eta, double stale_weight, int64_t epochs);
int mpa_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count, double scale, void* hip_stream);
int mpa_read_bandwidth(const void* buf, size_t bytes, int grid, int reps, void* hip_stream, double* gbps_out);
"""

_PROTO = re.compile(r"([A-Za-z_][\w \*]*?)\b(mpa_\w+)\s*\(([^;{]*?)\)\s*;", re.S)


def parse(text):
    """[(name, return type, [(param type, param name), ...])] of every mpa_* prototype in
    C source text (comments and preprocessor lines removed; the nwait typedef skipped)."""
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"#[^\n]*", "", text)
    out = []
    for m in _PROTO.finditer(text):
        ret, name, args = " ".join(m.group(1).split()), m.group(2), " ".join(m.group(3).split())
        if name == "mpa_nwait_fn" or ret.endswith("(*"):
            continue
        params = []
        if args not in ("", "void"):
            for a in args.split(","):
                a = a.strip()
                arr = re.search(r"\[\d*\]$", a)
                if arr:  # `double out[4]` is a pointer parameter
                    a = a[:arr.start()]
                    pm = re.match(r"(.*?)(\w+)$", a)
                    params.append((" ".join(pm.group(1).split()) + "*", pm.group(2)))
                    continue
                pm = re.match(r"(.*?)(\w+)$", a)
                params.append((" ".join(pm.group(1).replace("*", " * ").split()).replace(" *", "*"), pm.group(2)))
        out.append((name, ret.replace(" *", "*"), params))
    return out


def table():
    return parse(PROTOTYPES)


# C scalar types of the ABI
_SCALARS = {"int": ("c_int", "Cint"), "int64_t": ("c_int64", "Int64"), "uint64_t": ("c_uint64", "UInt64"),
            "uint32_t": ("c_uint32", "UInt32"), "size_t": ("c_size_t", "Csize_t"), "double": ("c_double", "Cdouble")}
# pointee of a typed return pointer
_POINTEES = {"int64_t": "Int64", "uint8_t": "UInt8", "double": "Cdouble", "int": "Cint", "char": "UInt8"}


def _base(t):
    return t.replace("const ", "").replace("*", "").strip()


def ctypes_type(t, is_return=False):
    """ctypes type of a C type: pointer PARAMETERS are c_void_p (they accept ints, arrays,
    byref and None alike); returned pointers are typed, strings are c_char_p."""
    import ctypes as C
    if t == "void":
        return None
    if t in ("const char*", "char*"):
        return C.c_char_p
    if t == "mpa_nwait_fn":
        return C.c_void_p
    if t.endswith("*"):
        if not is_return:
            return C.c_void_p
        base = _base(t)
        if t.count("*") == 1 and base in ("int64_t", "uint8_t", "double"):
            return C.POINTER({"int64_t": C.c_int64, "uint8_t": C.c_uint8, "double": C.c_double}[base])
        return C.c_void_p
    return getattr(C, _SCALARS[t][0])


def julia_type(t):
    """Julia ccall type of a C type."""
    if t == "void":
        return "Cvoid"
    if t in ("const char*", "char*"):
        return "Cstring"
    if t == "mpa_nwait_fn":
        return "Ptr{Cvoid}"
    if t.endswith("**"):
        inner = julia_type(t[:-1])
        return "Ptr{%s}" % inner
    if t.endswith("*"):
        base = _base(t)
        if base in ("mpa_pool", "mpa_comm", "void"):
            return "Ptr{Cvoid}"
        return "Ptr{%s}" % _POINTEES[base]
    return _SCALARS[t][1]


def ctypes_signatures():
    """(name, restype, argtypes) for every entry point: what `_capi.lib()` declares."""
    return [(name, ctypes_type(ret, True), [ctypes_type(t) for t, _ in params]) for name, ret, params in table()]
