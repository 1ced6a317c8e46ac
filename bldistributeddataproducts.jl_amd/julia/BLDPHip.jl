#=
BLDPHip.jl — the Julia side of the drop-in: `ccall` bindings to libbldp_hip
(include/bldp.h) for BLDistributedDataProducts.jl's WorkerFunctions.

UNTESTED HERE: Julia is absent from both the build container and the MI355X
box (probed), so this file is the binding a maintainer adds, exercised in this
repo only through the identical Python ctypes binding (_lib.py / tests/).
See INTEGRATION.md for the two-line patch to src/gbtworkerfunctions.jl.
=#
module BLDPHip

using Statistics: mean

export gpu_init, gpu_finalize, gpu_pin, gpu_unpin, gpu_fqav, gpu_reduce, gpu_kurtosis, gpu_band,
       gpu_comm_id, gpu_comm_init, gpu_comm_destroy, gpu_band_gather

const libbldp = get(ENV, "BLDP_LIB", joinpath(@__DIR__, "..", "libbldp_hip.so"))

# include/bldp.h BLDP_ABI_VERSION this binding is written against
const ABI_VERSION = 5
function __init__()
    v = ccall((:bldp_abi_version, libbldp), Cint, ())
    v == ABI_VERSION || error("libbldp_hip ABI version $v, BLDPHip expects $ABI_VERSION: rebuild it")
end

# bldp_dtype codes (include/bldp.h) and the element type of each code
const GPUElt = Union{Float32,Float64,UInt8,UInt16,UInt32,UInt64,Int8,Int16,Int32,Int64}
const ELTYPES = (Float32, Float64, UInt8, UInt16, UInt32, UInt64, Int8, Int16, Int32, Int64)
dtypecode(::Type{T}) where {T<:GPUElt} = Cint(findfirst(==(T), ELTYPES) - 1)

# fqavfunc values with a GPU implementation (README.md:192-195); anything
# else keeps the reference's host fqav.
opcode(f) = f === sum ? Cint(0) : f === mean ? Cint(1) : f === maximum ? Cint(2) :
            f === minimum ? Cint(3) : nothing

function lasterror()
    buf = Vector{UInt8}(undef, 1024)
    ccall((:bldp_last_error, libbldp), Cint, (Ptr{UInt8}, Csize_t), buf, length(buf))
    unsafe_string(pointer(buf))
end

function check(rc::Integer)
    rc == 0 && return nothing
    msg = lasterror()
    rc == -2 && throw(DimensionMismatch(msg))   # fqavby/tavby does not divide
    rc == -6 && throw(BoundsError(msg))         # window outside the array
    rc == -1 && throw(ArgumentError(msg))
    rc == -8 && throw(SystemError(msg))         # a file read failed or ended early
    error("libbldp_hip error $rc: $msg")
end

"""
    gpu_init(devs=nothing)

bldp_init: validate the GPUs (gfx950), create their worker streams and warm
host-staging pipelines, enable xGMI peer access between them.  Called once per
worker process after `GBT.setupworkers` (src/gbt.jl:12-46) has started it;
optional, since every entry point initialises what it needs on first use.
`nothing` selects every visible device."""
function gpu_init(devs::Union{Nothing,AbstractVector{<:Integer}}=nothing)
    if devs === nothing
        check(ccall((:bldp_init, libbldp), Cint, (Cint, Ptr{Cint}), 0, C_NULL))
    else
        d = Cint.(collect(devs))
        GC.@preserve d check(ccall((:bldp_init, libbldp), Cint, (Cint, Ptr{Cint}), length(d), d))
    end
    nothing
end

"bldp_finalize: drain the devices and free every library-owned resource."
gpu_finalize() = (check(ccall((:bldp_finalize, libbldp), Cint, ())); nothing)

"""
    gpu_pin(A::Array) / gpu_unpin(A::Array)

Page-lock a long-lived host array (bldp_host_register) so gpu_reduce and
gpu_kurtosis copy it at full PCIe rate; the caller keeps `A` alive meanwhile."""
gpu_pin(A::Array) = (check(ccall((:bldp_host_register, libbldp), Cint, (Ptr{Cvoid}, Csize_t),
                                 A, sizeof(A))); A)
gpu_unpin(A::Array) = (check(ccall((:bldp_host_unregister, libbldp), Cint, (Ptr{Cvoid},), A));
                       A)

# Julia index -> (0-based start, count, step) on an axis of length n
axiswin(::Colon, n) = (0, n, 1)
axiswin(i::Integer, n) = (i - 1, 1, 1)                      # sanitizeidxs: i -> i:i
axiswin(r::AbstractRange{<:Integer}, n) = (first(r) - 1, length(r), step(r))

function window(idxs::Tuple, sz)
    @assert length(idxs) == 3 "idxs must have exactly three indices"
    all(i -> i isa Colon, idxs) && return Ptr{Int64}(C_NULL)
    Int64[x for ax in 1:3 for x in axiswin(idxs[ax], sz[ax])]
end

"""
    gpu_reduce(A::Array{Float32,3}, fqavby, tavby=1; f=sum, idxs=(:,:,:), dev=0)

`fqav(A[idxs...], fqavby; f)` fused with the same reduction over `tavby`
spectra, computed on GPU `dev` (bldp_reduce_host_f32)."""
function gpu_reduce(A::Array{Float32,3}, fqavby::Integer, tavby::Integer=1;
                    f=sum, idxs::Tuple=(:, :, :), dev::Integer=0)
    op = opcode(f)
    op === nothing && throw(ArgumentError("no GPU kernel for $f"))
    win = window(idxs, size(A))
    shp = zeros(Int64, 3)
    GC.@preserve win check(ccall((:bldp_reduce_shape, libbldp), Cint,
        (Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Ptr{Int64}),
        size(A, 1), size(A, 2), size(A, 3), win, fqavby, tavby, shp))
    out = Array{Float32,3}(undef, shp...)
    GC.@preserve A win out check(ccall((:bldp_reduce_host_f32, libbldp), Cint,
        (Cint, Ptr{Float32}, Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Cint, Ptr{Float32}),
        dev, A, size(A, 1), size(A, 2), size(A, 3), win, fqavby, tavby, op, out))
    out
end

"""
    gpu_reduce(A::Array{T,3}, fqavby, tavby=1; f=sum, idxs=(:,:,:), dev=0) for T other than Float32

The same for integer and Float64 data (SIGPROC nbits 8 / 16 mmaps to UInt8 /
UInt16, src/gbtworkerfunctions.jl:173), with fqav's Julia result type:
bldp_reduce_out_dtype (sum widened to (U)Int64 exactly, mean Float64,
maximum / minimum the input type), reduced on GPU `dev` (bldp_reduce_host)."""
function gpu_reduce(A::Array{T,3}, fqavby::Integer, tavby::Integer=1;
                    f=sum, idxs::Tuple=(:, :, :), dev::Integer=0) where {T<:GPUElt}
    op = opcode(f)
    op === nothing && throw(ArgumentError("no GPU kernel for $f"))
    od = ccall((:bldp_reduce_out_dtype, libbldp), Cint, (Cint, Cint), dtypecode(T), op)
    od < 0 && check(od)
    win = window(idxs, size(A))
    shp = zeros(Int64, 3)
    GC.@preserve win check(ccall((:bldp_reduce_shape, libbldp), Cint,
        (Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Ptr{Int64}),
        size(A, 1), size(A, 2), size(A, 3), win, fqavby, tavby, shp))
    out = Array{ELTYPES[od + 1],3}(undef, shp...)
    GC.@preserve A win out check(ccall((:bldp_reduce_host, libbldp), Cint,
        (Cint, Cint, Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Cint, Ptr{Cvoid}),
        dev, dtypecode(T), A, size(A, 1), size(A, 2), size(A, 3), win, fqavby, tavby, op, out))
    out
end

"""
    gpu_fqav(A, n; f=sum, tavby=1)

Drop-in for `fqav(A, n; f)` (src/gbtworkerfunctions.jl:16-20): same
pass-through for `n <= 1`, same DimensionMismatch, GPU for sum/mean/maximum/
minimum, the reference's host code for any other `f`."""
function gpu_fqav(A, n::Integer; f=sum, tavby::Integer=1, dev::Integer=0)
    (n <= 1 && tavby <= 1) && return A
    if A isa Array{<:GPUElt,3} && opcode(f) !== nothing
        return gpu_reduce(A, n, tavby; f, dev)
    end
    tavby <= 1 || throw(ArgumentError("tavby needs a 3-D array and sum/mean/max/min"))
    sz = (n, :, size(A)[2:end]...)
    dropdims(f(reshape(A, sz), dims=1), dims=1)
end

"""
    gpu_kurtosis(A::Array{Float32,3}; idxs=(:,:,:), dev=0) -> Matrix{Float64}

getkurtosis' per-(channel, IF) excess kurtosis over time
(src/gbtworkerfunctions.jl:197-202), computed on GPU `dev`
(bldp_kurtosis_host_f32: window staged on the device, StatsBase recipe,
Float64 result)."""
function gpu_kurtosis(A::Array{Float32,3}; idxs::Tuple=(:, :, :), dev::Integer=0)
    win = window(idxs, size(A))
    shp = zeros(Int64, 3)
    GC.@preserve win check(ccall((:bldp_reduce_shape, libbldp), Cint,
        (Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Ptr{Int64}),
        size(A, 1), size(A, 2), size(A, 3), win, 1, 1, shp))
    out = Matrix{Float64}(undef, shp[1], shp[2])
    GC.@preserve A win out check(ccall((:bldp_kurtosis_host_f32, libbldp), Cint,
        (Cint, Ptr{Float32}, Int64, Int64, Int64, Ptr{Int64}, Ptr{Float64}),
        dev, A, size(A, 1), size(A, 2), size(A, 3), win, out))
    out
end

"""
    gpu_kurtosis(A::Array{T,3}; idxs=(:,:,:), dev=0) for T other than Float32

StatsBase.kurtosis of integer or Float64 rows (Float64 throughout: Base.sum's
pairwise mean, sequential moments), on GPU `dev` (bldp_kurtosis_host)."""
function gpu_kurtosis(A::Array{T,3}; idxs::Tuple=(:, :, :), dev::Integer=0) where {T<:GPUElt}
    win = window(idxs, size(A))
    shp = zeros(Int64, 3)
    GC.@preserve win check(ccall((:bldp_reduce_shape, libbldp), Cint,
        (Int64, Int64, Int64, Ptr{Int64}, Int64, Int64, Ptr{Int64}),
        size(A, 1), size(A, 2), size(A, 3), win, 1, 1, shp))
    out = Matrix{Float64}(undef, shp[1], shp[2])
    GC.@preserve A win out check(ccall((:bldp_kurtosis_host, libbldp), Cint,
        (Cint, Cint, Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Int64}, Ptr{Float64}),
        dev, dtypecode(T), A, size(A, 1), size(A, 2), size(A, 3), win, out))
    out
end

"""
    gpu_band(parts) -> Array{Float32,3}

`reduce(vcat, parts)` of per-bank results in bank order (src/gbt.jl:103):
what `GBT.getband` returns after `fetch.(futures)`."""
gpu_band(parts) = reduce(vcat, parts)

# ---------------------------------------------------------------------------
# Band stitch across worker processes, one GPU each, over RCCL (xGMI): the
# device-side replacement of GBT.getdata's fetch of every worker's result
# (src/gbt.jl:75-78).  The 128-byte id travels between workers through
# Distributed (e.g. `remotecall_fetch(gpu_comm_id, first(workers))`).

"RCCL unique id for a new band communicator (call on one worker)."
function gpu_comm_id()
    id = zeros(UInt8, 128)
    check(ccall((:bldp_comm_id, libbldp), Cint, (Ptr{UInt8},), id))
    id
end

"Join the band communicator (collective over all `nranks` workers)."
function gpu_comm_init(id::Vector{UInt8}, nranks::Integer, rank::Integer; dev::Integer=0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:bldp_comm_init, libbldp), Cint, (Cint, Cint, Cint, Ptr{UInt8}, Ptr{Ptr{Cvoid}}),
                dev, nranks, rank, id, h))
    h[]
end

gpu_comm_destroy(comm::Ptr{Cvoid}) =
    (check(ccall((:bldp_comm_destroy, libbldp), Cint, (Ptr{Cvoid},), comm)); nothing)

"""
    gpu_band_gather(comm, slice::Ptr{Float32}, count, gathered::Ptr{Float32}; root=0, stream=C_NULL)

ncclGather of every worker's reduced slice (a device buffer of `count`
Float32, its banks in vcat order) into `gathered` (nranks*count) on `root`,
rank-major; then `bldp_stitch_f32` when the product has more than one
(IF, time) row.  Device pointers; asynchronous on `stream`."""
gpu_band_gather(comm::Ptr{Cvoid}, slice::Ptr{Float32}, count::Integer, gathered::Ptr{Float32};
                root::Integer=0, stream::Ptr{Cvoid}=C_NULL) =
    (check(ccall((:bldp_band_gather_f32, libbldp), Cint,
                 (Ptr{Cvoid}, Cint, Ptr{Float32}, Int64, Ptr{Float32}, Ptr{Cvoid}),
                 comm, root, slice, count, gathered, stream)); nothing)

end # module
