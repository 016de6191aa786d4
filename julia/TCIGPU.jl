# TCIGPU.jl -- the Julia side of the drop-in: TensorCrossInterpolation.jl's TCI2 hot path on an
# MI355X through libtci_hip.so (include/tci_hip.h). Load it next to the reference package:
#
#     import TensorCrossInterpolation as TCI
#     include("julia/TCIGPU.jl"); using .TCIGPU
#     ctx = TCIGPU.Ctx(0)
#     f = TCIGPU.GPUBatchEvaluator(ctx, TCIGPU.TCI_F_LORENTZ, [1.0], fill(10, 8), v -> 1 / (1 + v' * v))
#     tci, ranks, errors = TCI.crossinterpolate2(Float64, f, fill(10, 8); tolerance=1e-8)
#
# The extension point is the reference's own plugin type, `BatchEvaluator{T}`
# (src/cachedtensortrain.jl:31, contract in docs/src/index.md:174-243): `crossinterpolate2`'s `f`
# flows unchanged through optimize! -> sweep2site! -> updatepivots! / setsitetensor!, so the methods
# below, specialised on the evaluator types of this module, replace the hot path and leave the user
# API untouched (INTEGRATION.md explains each binding).
#
# STATUS: unverified at runtime -- Julia is not installed in the build image. Every `ccall` signature
# here is checked mechanically against include/tci_hip.h by tests/test_julia_shim.py (argument
# count, pointer-ness and scalar widths), and the same entry points are exercised through ctypes by
# the Python host mirror (tensorcrossinterpolation.jl_amd/tci_amd) in tests/.
module TCIGPU

import TensorCrossInterpolation as TCI
using TensorCrossInterpolation: TensorCI2, MultiIndex, kronecker, updateerrors!, invalidatesitetensors!

export Ctx, GPUBatchEvaluator, HostFunctionEvaluator, GPUContraction, GPUComm, rrlu_sharded

const libtci = get(ENV, "TCI_HIP_LIB", "libtci_hip.so")

# error codes (include/tci_hip.h)
const TCI_OK, TCI_ERR_ARG, TCI_ERR_NAN, TCI_ERR_NONSQ, TCI_ERR_DEVICE, TCI_ERR_NOMEM, TCI_ERR_HOST = 0, 1, 2, 3, 4, 5, 6
# integrand kinds (include/tci_hip.h TCI_F_*)
const TCI_F_SUM, TCI_F_LORENTZ, TCI_F_TABLE, TCI_F_GAUSS, TCI_F_GAUSSMIX, TCI_F_QOSC = 0, 1, 2, 3, 4, 5
const TCI_F_QEXP, TCI_F_TT, TCI_F_CP, TCI_F_MPO, TCI_F_HOST, TCI_F_C128 = 6, 7, 8, 9, 10, 11

# ------------------------------------------------------------------ context and errors
mutable struct Ctx
    h::Ptr{Cvoid}
end

function Ctx(device::Integer=0)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    st = ccall((:tci_ctx_create, libtci), Cint, (Cint, Ref{Ptr{Cvoid}}), device, r)
    st == TCI_OK || error("tci_ctx_create failed ($st): no MI355X visible?")
    c = Ctx(r[])
    finalizer(c) do c
        c.h == C_NULL || ccall((:tci_ctx_destroy, libtci), Cint, (Ptr{Cvoid},), c.h)
        c.h = C_NULL
    end
    return c
end

const DEFAULT_CTX = Ref{Union{Nothing,Ctx}}(nothing)
default_ctx() = something(DEFAULT_CTX[], begin DEFAULT_CTX[] = Ctx(parse(Int, get(ENV, "LOCAL_RANK", "0"))) end)

# an exception raised by the user's f inside a host batch callback, rethrown after TCI_ERR_HOST
const HOST_ERROR = Ref{Any}(nothing)

function check(c::Ctx, st)
    st == TCI_OK && return nothing
    if st == TCI_ERR_HOST && HOST_ERROR[] !== nothing
        e = HOST_ERROR[]
        HOST_ERROR[] = nothing
        throw(e)
    end
    msg = unsafe_string(ccall((:tci_last_error, libtci), Cstring, (Ptr{Cvoid},), c.h))
    st == TCI_ERR_ARG && throw(ArgumentError(msg))
    error(msg)   # "lu.L contains NaNs" etc.: the reference's own text (matrixlu.jl:376-381)
end

synchronize(c::Ctx) = check(c, ccall((:tci_ctx_synchronize, libtci), Cint, (Ptr{Cvoid},), c.h))

# tuning switches (results are bitwise the same either way; they exist for A/B timing)
set_shadow!(c::Ctx, on::Bool) = check(c, ccall((:tci_set_rrlu_shadow, libtci), Cint, (Ptr{Cvoid}, Cint), c.h, on))
set_c128_shadow!(c::Ctx, on::Bool) = check(c, ccall((:tci_set_c128_shadow, libtci), Cint, (Ptr{Cvoid}, Cint), c.h, on))
set_rrlu_epochs!(c::Ctx, e::Integer) = check(c, ccall((:tci_set_rrlu_epochs, libtci), Cint, (Ptr{Cvoid}, Cint), c.h, e))
set_shard_exchange!(c::Ctx, mode::Integer) =
    check(c, ccall((:tci_set_shard_exchange, libtci), Cint, (Ptr{Cvoid}, Cint), c.h, mode))
last_shard_exchange(c::Ctx) = ccall((:tci_last_shard_exchange, libtci), Cint, (Ptr{Cvoid},), c.h)
shadow_bytes() = ccall((:tci_rrlu_shadow_bytes, libtci), Cint, ())

# entries of a Vector{MultiIndex} as a row-major Int32 table (1-based, as in Julia)
table(S::Vector{MultiIndex}) = isempty(S) ? Int32[] : Int32.(reduce(vcat, S))

# ------------------------------------------------------------------ evaluators (BatchEvaluator plugins)
abstract type DeviceEvaluator <: TCI.BatchEvaluator{Float64} end

# An integrand from the device catalog (TCI_F_*): the batch, max|Pi|, the rrLU and the site-tensor
# solves all run on the device. hostf: single-point evaluation (the global pivot search,
# tensorci2.jl:440, and the reference's initial maxsamplevalue).
mutable struct GPUBatchEvaluator <: DeviceEvaluator
    ctx::Ctx
    h::Ptr{Cvoid}
    localdims::Vector{Int}
    hostf::Function
end

function GPUBatchEvaluator(ctx::Ctx, kind::Integer, params::Vector{Float64}, localdims::Vector{Int}, hostf)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    ld = Int32.(localdims)
    check(ctx, ccall((:tci_func_create, libtci), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Int64, Ptr{Int32}, Int32, Ref{Ptr{Cvoid}}),
        ctx.h, kind, params, length(params), ld, length(ld), r))
    f = GPUBatchEvaluator(ctx, r[], localdims, hostf)
    finalizer(f) do f
        f.h == C_NULL || ccall((:tci_func_destroy, libtci), Cint, (Ptr{Cvoid},), f.h)
        f.h = C_NULL
    end
    return f
end

(f::GPUBatchEvaluator)(x::MultiIndex) = f.hostf(x)

# The user's own f (any closure) or BatchEvaluator{Float64}: evaluated on the host by a callback
# (TCI_F_HOST), everything after the batch on the device. The evaluator travels as the `user`
# pointer, so the callback is one static @cfunction.
mutable struct HostFunctionEvaluator{F} <: DeviceEvaluator
    ctx::Ctx
    h::Ptr{Cvoid}
    f::F
    localdims::Vector{Int}
end

(e::HostFunctionEvaluator)(x::MultiIndex) = e.f(x)

function _host_batch(user::Ptr{Cvoid}, pI::Ptr{Int32}, m::Int64, nl::Int32, pJ::Ptr{Int32}, n::Int64,
                     nr::Int32, M::Int32, out::Ptr{Float64}, ldo::Int64)::Cint
    e = unsafe_pointer_to_objref(user)::HostFunctionEvaluator
    try
        I = [Int.(unsafe_wrap(Vector{Int32}, pI + 4nl * (i - 1), Int(nl))) for i in 1:m]
        J = [Int.(unsafe_wrap(Vector{Int32}, pJ + 4nr * (j - 1), Int(nr))) for j in 1:n]
        # the generic loop (batcheval.jl:131-175), or the user's BatchEvaluator / ThreadedBatchEvaluator
        vals = TCI._batchevaluate_dispatch(Float64, e.f, e.localdims, I, J, Val(Int(M)))
        R = div(length(vals), max(n, 1))
        dst = unsafe_wrap(Matrix{Float64}, out, (Int(ldo), Int(n)))
        dst[1:R, :] .= reshape(vals, R, n)
        return Cint(0)
    catch err
        HOST_ERROR[] = err
        return Cint(1)
    end
end

function HostFunctionEvaluator(ctx::Ctx, f, localdims::Vector{Int})
    e = HostFunctionEvaluator(ctx, C_NULL, f, localdims)
    cb = @cfunction(_host_batch, Cint, (Ptr{Cvoid}, Ptr{Int32}, Int64, Int32, Ptr{Int32}, Int64, Int32, Int32,
                                        Ptr{Float64}, Int64))
    r = Ref{Ptr{Cvoid}}(C_NULL)
    ld = Int32.(localdims)
    check(ctx, ccall((:tci_func_create_host, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Any, Ptr{Int32}, Int32, Ref{Ptr{Cvoid}}),
        ctx.h, cb, e, ld, length(ld), r))   # `Any`: the object's address (e stays rooted by the caller)
    e.h = r[]
    finalizer(e) do e
        e.h == C_NULL || ccall((:tci_func_destroy, libtci), Cint, (Ptr{Cvoid},), e.h)
        e.h = C_NULL
    end
    return e
end

# BatchEvaluator contract (docs/src/index.md:174-243): an Array{Float64, M + 2}
function (f::DeviceEvaluator)(I::Vector{MultiIndex}, J::Vector{MultiIndex}, ::Val{M}) where {M}
    nl = isempty(I) ? 0 : length(first(I))
    nr = isempty(J) ? 0 : length(first(J))
    D = prod(f.localdims[nl+1:nl+M]; init=1)
    out = Array{Float64}(undef, length(I), f.localdims[nl+1:nl+M]..., length(J))
    isempty(out) && return out
    mx = Ref(0.0)
    check(f.ctx, ccall((:tci_batcheval_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Int32}, Int64, Int32, Ptr{Int32}, Int64, Int32, Int32,
         Ptr{Float64}, Int64, Ref{Float64}),
        f.ctx.h, f.h, table(I), length(I), nl, table(J), length(J), nr, M, out, length(I) * D, mx))
    return out
end

# Contraction(A, B) of two tensor-train operators (contraction.jl:60-152) as integrand TCI_F_MPO:
# params = [N, per site (ra, d1, d2, ra', rb, d3, rb', offA, offB), cores A_t (ra,d1,d2,ra'), B_t (rb,d2,d3,rb')]
function GPUContraction(ctx::Ctx, a::TCI.TensorTrain{Float64,4}, b::TCI.TensorTrain{Float64,4})
    hdr = Float64[length(a)]
    blob = Float64[]
    for (A, B) in zip(TCI.sitetensors(a), TCI.sitetensors(b))
        offA = length(blob); append!(blob, vec(A))
        offB = length(blob); append!(blob, vec(B))
        append!(hdr, [size(A, 1), size(A, 2), size(A, 3), size(A, 4), size(B, 1), size(B, 3), size(B, 4), offA, offB])
    end
    localdims = [size(A, 2) * size(B, 3) for (A, B) in zip(TCI.sitetensors(a), TCI.sitetensors(b))]
    cab = TCI.Contraction(a, b)   # single points f(x) on the host
    return GPUBatchEvaluator(ctx, TCI_F_MPO, vcat(hdr, blob), localdims, x -> cab(x))
end

# A ComplexF64 integrand as sums of real parts (Re f = sum(parts_re), Im f = sum(parts_im)): the
# realified complex contraction (INTEGRATION.md), consumed by tci_update_pivots_c128_h
function complex_integrand(ctx::Ctx, parts_re::Vector{Ptr{Cvoid}}, parts_im::Vector{Ptr{Cvoid}})
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ctx, ccall((:tci_func_create_c128, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Int32, Ptr{Ptr{Cvoid}}, Int32, Ref{Ptr{Cvoid}}),
        ctx.h, parts_re, length(parts_re), parts_im, length(parts_im), out))
    return out[]
end

# ------------------------------------------------------------------ the TCI2 hot path
# updatepivots! :full branch (tensorci2.jl:825-930) with Pi device-resident: index tables in, pivot
# indices, pivot errors, max|Pi| and (when observable) the MatrixLUCI factors out
function TCI.updatepivots!(tci::TensorCI2{Float64}, b::Int, f::DeviceEvaluator, leftorthogonal::Bool;
        reltol::Float64=1e-14, abstol::Float64=0.0, maxbonddim::Int=typemax(Int),
        sweepdirection::Symbol=:forward, pivotsearch::Symbol=:full, verbosity::Int=0,
        extraIset::Vector{MultiIndex}=MultiIndex[], extraJset::Vector{MultiIndex}=MultiIndex[])
    pivotsearch === :full || throw(ArgumentError("the device evaluators support pivotsearch=:full"))
    invalidatesitetensors!(tci)
    Icomb = union(kronecker(tci.Iset[b], tci.localdims[b]), extraIset)
    Jcomb = union(kronecker(tci.localdims[b+1], tci.Jset[b+1]), extraJset)
    m, n = length(Icomb), length(Jcomb)
    nl, nr = b, length(tci.localdims) - b
    r = max(min(maxbonddim, m, n), 0)
    rowidx = Vector{Int64}(undef, max(r, 1)); colidx = Vector{Int64}(undef, max(r, 1))
    perr = Vector{Float64}(undef, r + 1); np = Ref{Int64}(0); mx = Ref(0.0)
    wantf = isempty(extraIset) && isempty(extraJset)
    left = wantf ? Matrix{Float64}(undef, m, max(r, 1)) : Matrix{Float64}(undef, 0, 0)
    right = wantf ? Vector{Float64}(undef, max(r, 1) * n) : Float64[]   # np x n, ld np
    check(f.ctx, ccall((:tci_update_pivots_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Int32}, Int64, Int32, Ptr{Int32}, Int64, Int32, Int64,
         Float64, Float64, Cint, Cint, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ref{Int64},
         Ref{Float64}, Ptr{Float64}, Ptr{Float64}),
        f.ctx.h, f.h, table(Icomb), m, nl, table(Jcomb), n, nr, maxbonddim,
        reltol, abstol, leftorthogonal, wantf, rowidx, colidx, perr, np, mx, left, right))
    k = Int(np[])
    tci.maxsamplevalue = max(tci.maxsamplevalue, mx[])   # updatemaxsample!, tensorci2.jl:636-638
    tci.Iset[b+1] = Icomb[rowidx[1:k]]
    tci.Jset[b] = Jcomb[colidx[1:k]]
    if wantf
        TCI.setsitetensor!(tci, b, left[:, 1:k])
        TCI.setsitetensor!(tci, b + 1, reshape(right[1:k*n], k, n))
    end
    updateerrors!(tci, b, perr[1:k+1])
    return nothing
end

# setsitetensor!(tci, f, b) (tensorci2.jl:599-629): T = Pi1 * P^-1 solved on the device
function TCI.setsitetensor!(tci::TensorCI2{Float64}, f::DeviceEvaluator, b::Int; leftorthogonal=true)
    leftorthogonal || error("leftorthogonal==false is not supported!")
    Ib, Jb = tci.Iset[b], tci.Jset[b]
    last = b == length(tci)
    Inext = last ? MultiIndex[] : tci.Iset[b+1]
    T = Matrix{Float64}(undef, length(Ib) * tci.localdims[b], length(Jb))
    mx = Ref(0.0)
    st = ccall((:tci_sitetensor_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Int32}, Int64, Int32, Ptr{Int32}, Int64, Int32,
         Ptr{Int32}, Int64, Ptr{Float64}, Ref{Float64}),
        f.ctx.h, f.h, table(Ib), length(Ib), b - 1, table(Jb), length(Jb), length(tci) - b,
        last ? Int32[] : table(Inext), length(Inext), T, mx)
    st == TCI_ERR_NONSQ && error("Pivot matrix at bond $(b) is not square!")
    check(f.ctx, st)
    tci.maxsamplevalue = max(tci.maxsamplevalue, mx[])
    tci.sitetensors[b] = reshape(T, length(Ib), tci.localdims[b], :)
    return tci.sitetensors[b]
end

# ------------------------------------------------------------------ whole sweeps on the device
# The native sweep driver (tci_tci2_*): sweep2site!'s per-bond loop (tensorci2.jl:1195-1258) --
# kronecker products, first-seen union, the 2-site update, updatemaxsample!, updateerrors! -- in
# C++ and, for staged catalog kinds whose bonds fit one workgroup, in ONE device launch.
mutable struct DeviceState
    h::Ptr{Cvoid}
end

function DeviceState(ctx::Ctx, localdims::Vector{Int})
    r = Ref{Ptr{Cvoid}}(C_NULL)
    ld = Int32.(localdims)
    check(ctx, ccall((:tci_tci2_create, libtci), Cint, (Ptr{Cvoid}, Int32, Ptr{Int32}, Ref{Ptr{Cvoid}}),
                     ctx.h, length(ld), ld, r))
    s = DeviceState(r[])
    finalizer(s) do s
        s.h == C_NULL || ccall((:tci_tci2_destroy, libtci), Cint, (Ptr{Cvoid},), s.h)
        s.h = C_NULL
    end
    return s
end

# which: 0 Iset, 1 Jset -- packed as counts (one per site) and the entries back to back
function push_sets!(ctx::Ctx, s::DeviceState, tci::TensorCI2{Float64})
    for (which, sets) in ((0, tci.Iset), (1, tci.Jset))
        counts = Int64[length(S) for S in sets]
        packed = isempty(sets) ? Int32[] : reduce(vcat, [table(S) for S in sets])
        check(ctx, ccall((:tci_tci2_set_sets, libtci), Cint, (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Int32}),
                         s.h, which, counts, packed))
    end
    # which 2 / 3: the last sweep's sets (Iset_history[end] / Jset_history[end]), the first-seen
    # union's second operand when the sweep is not strictly nested (tensorci2.jl:1214-1216)
    if !isempty(tci.Iset_history)
        for (which, sets) in ((2, tci.Iset_history[end]), (3, tci.Jset_history[end]))
            counts = Int64[length(S) for S in sets]
            packed = isempty(sets) ? Int32[] : reduce(vcat, [table(S) for S in sets])
            check(ctx, ccall((:tci_tci2_set_sets, libtci), Cint, (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Int32}),
                             s.h, which, counts, packed))
        end
    end
    pe = tci.pivoterrors
    check(ctx, ccall((:tci_tci2_set_errors, libtci), Cint, (Ptr{Cvoid}, Float64, Ptr{Float64}, Ptr{Float64}, Int64),
                     s.h, tci.maxsamplevalue, tci.bonderrors, pe, length(pe)))
end

function pull_sets!(ctx::Ctx, s::DeviceState, tci::TensorCI2{Float64}; history::Bool=false)
    L = length(tci.localdims)
    if history   # the sweep's own history entries (which 2 / 3) appended as the reference's loop does
        push!(tci.Iset_history, [MultiIndex[] for _ in 1:L])
        push!(tci.Jset_history, [MultiIndex[] for _ in 1:L])
    end
    banks = ((0, tci.Iset, p -> p - 1), (1, tci.Jset, p -> L - p))
    history && (banks = (banks..., (2, tci.Iset_history[end], p -> p - 1), (3, tci.Jset_history[end], p -> L - p)))
    for (which, sets, width) in banks
        counts = Vector{Int64}(undef, L)
        cap = Int64(1 << 24)
        packed = Vector{Int32}(undef, cap)
        check(ctx, ccall((:tci_tci2_get_sets, libtci), Cint, (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Int32}, Int64),
                         s.h, which, counts, packed, cap))
        o = 0
        for p in 1:L
            w = width(p)
            sets[p] = [Int.(packed[o+w*(i-1)+1:o+w*i]) for i in 1:counts[p]]
            o += w * counts[p]
        end
    end
    ms = Ref(0.0); npe = Ref{Int64}(0)
    pe = Vector{Float64}(undef, 1 << 16)
    check(ctx, ccall((:tci_tci2_errors, libtci), Cint, (Ptr{Cvoid}, Ref{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                     s.h, ms, tci.bonderrors, pe, length(pe), npe))
    tci.maxsamplevalue = ms[]
    resize!(tci.pivoterrors, npe[])
    tci.pivoterrors .= pe[1:npe[]]
end

# sweep2site!(tci, f, niter; ...) for a device integrand; returns false (state untouched) when the
# driver cannot take it, and the reference's method then runs
function sweep2site_device!(tci::TensorCI2{Float64}, f::GPUBatchEvaluator, niter::Int; iter1::Int=1,
        abstol::Float64=1e-8, maxbonddim::Int=typemax(Int), sweepstrategy::Symbol=:backandforth,
        strictlynested::Bool=false)
    strategy = sweepstrategy === :backandforth ? 0 : sweepstrategy === :forward ? 1 : 2
    s = DeviceState(f.ctx, tci.localdims)
    push_sets!(f.ctx, s, tci)
    check(f.ctx, ccall((:tci_tci2_sweep2site, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Int32, Int32, Float64, Int64, Int32, Int32),
        s.h, f.h, niter, iter1, abstol, maxbonddim, strategy, strictlynested))
    pull_sets!(f.ctx, s, tci; history=!strictlynested)
    invalidatesitetensors!(tci)
    return true
end

# sweep1site! (tensorci2.jl:659-725) in one device launch when every bond fits; false otherwise
function sweep1site_device!(tci::TensorCI2{Float64}, f::GPUBatchEvaluator, sweepdirection::Symbol=:forward;
        reltol::Float64=1e-14, abstol::Float64=0.0, maxbonddim::Int=typemax(Int), updatetensors::Bool=true)
    s = DeviceState(f.ctx, tci.localdims)
    push_sets!(f.ctx, s, tci)
    tens = Vector{Float64}(undef, length(tci) * 16384)
    offs = zeros(Int64, 2 * length(tci))
    handled = Ref{Cint}(0)
    check(f.ctx, ccall((:tci_tci2_sweep1site, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Int32, Float64, Float64, Int64, Int32, Ptr{Float64}, Int64, Ptr{Int64}, Ref{Cint}),
        s.h, f.h, sweepdirection === :forward, reltol, abstol, maxbonddim, updatetensors,
        tens, length(tens), offs, handled))
    handled[] == 1 || return false
    pull_sets!(f.ctx, s, tci)
    if updatetensors
        for p in 1:length(tci)
            o, len = offs[2p-1], offs[2p]
            len > 0 && (tci.sitetensors[p] = reshape(tens[o+1:o+len], length(tci.Iset[p]), tci.localdims[p], :))
        end
    end
    return true
end

# fillsitetensors! (globalsearch.jl:202-208) with every site tensor solved (setsitetensor!,
# tensorci2.jl:599-629) in one device launch; false when the device path cannot take it
function fillsitetensors_device!(tci::TensorCI2{Float64}, f::GPUBatchEvaluator)
    s = DeviceState(f.ctx, tci.localdims)
    push_sets!(f.ctx, s, tci)
    tens = Vector{Float64}(undef, length(tci) * 16384)
    offs = zeros(Int64, 2 * length(tci))
    handled = Ref{Cint}(0)
    check(f.ctx, ccall((:tci_tci2_fill_solve, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Int64}, Ref{Cint}),
        s.h, f.h, tens, length(tens), offs, handled))
    handled[] == 1 || return false
    ms = Ref(0.0)
    check(f.ctx, ccall((:tci_tci2_errors, libtci), Cint, (Ptr{Cvoid}, Ref{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Int64}),
                       s.h, ms, C_NULL, C_NULL, 0, C_NULL))
    tci.maxsamplevalue = ms[]
    for p in 1:length(tci)
        o, len = offs[2p-1], offs[2p]
        tci.sitetensors[p] = reshape(tens[o+1:o+len], length(tci.Iset[p]), tci.localdims[p], :)
    end
    return true
end

# ------------------------------------------------------------------ rrLU / MatrixLUCI
# rrlu(A; ...) (matrixlu.jl:455-463) for Float64 and ComplexF64 (interleaved, Julia's own layout)
function device_rrlu(A::Matrix{Float64}; maxrank::Int=typemax(Int), reltol::Number=1e-14,
        abstol::Number=0.0, leftorthogonal::Bool=true, ctx::Ctx=default_ctx())
    m, n = size(A); mr = max(min(maxrank, m, n), 0)
    rp = Vector{Int64}(undef, m); cp = Vector{Int64}(undef, n)
    L = Matrix{Float64}(undef, m, max(mr, 1)); U = Matrix{Float64}(undef, max(mr, 1), n)
    np = Ref{Int64}(0); err = Ref{Float64}(0.0)
    check(ctx, ccall((:tci_rrlu_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Int64, Int64, Float64, Float64, Cint,
         Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}, Ref{Float64}),
        ctx.h, A, m, n, m, maxrank, reltol, abstol, leftorthogonal, rp, cp, L, U, max(mr, 1), np, err))
    k = Int(np[])
    return TCI.rrLU(Int.(rp), Int.(cp), L[:, 1:k], U[1:k, :], leftorthogonal, k, err[])
end

function device_rrlu(A::Matrix{ComplexF64}; maxrank::Int=typemax(Int), reltol::Number=1e-14,
        abstol::Number=0.0, leftorthogonal::Bool=true, ctx::Ctx=default_ctx())
    m, n = size(A); mr = max(min(maxrank, m, n), 0)
    rp = Vector{Int64}(undef, m); cp = Vector{Int64}(undef, n)
    L = Matrix{ComplexF64}(undef, m, max(mr, 1)); U = Matrix{ComplexF64}(undef, max(mr, 1), n)
    np = Ref{Int64}(0); err = Ref{Float64}(0.0)
    GC.@preserve A L U check(ctx, ccall((:tci_rrlu_c128_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{ComplexF64}, Int64, Int64, Int64, Int64, Float64, Float64, Cint,
         Ptr{Int64}, Ptr{Int64}, Ptr{ComplexF64}, Ptr{ComplexF64}, Int64, Ref{Int64}, Ref{Float64}, Ptr{Float64}),
        ctx.h, A, m, n, m, maxrank, reltol, abstol, leftorthogonal, rp, cp, L, U, max(mr, 1), np, err, C_NULL))
    k = Int(np[])
    return TCI.rrLU(Int.(rp), Int.(cp), L[:, 1:k], U[1:k, :], leftorthogonal, k, err[])
end

# MatrixLUCI(A) factors (matrixluci.jl:161-283): pivot indices, pivot errors, left and right
function device_luci(A::Matrix{Float64}; maxrank::Int=typemax(Int), reltol::Number=1e-14,
        abstol::Number=0.0, leftorthogonal::Bool=true, ctx::Ctx=default_ctx())
    m, n = size(A); mr = max(min(maxrank, m, n), 0)
    ri = Vector{Int64}(undef, max(mr, 1)); ci = Vector{Int64}(undef, max(mr, 1))
    pe = Vector{Float64}(undef, mr + 1)
    left = Matrix{Float64}(undef, m, max(mr, 1)); right = Vector{Float64}(undef, max(mr, 1) * n)
    np = Ref{Int64}(0)
    check(ctx, ccall((:tci_luci_h, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Int64, Int64, Float64, Float64, Cint,
         Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Int64}),
        ctx.h, A, m, n, m, maxrank, reltol, abstol, leftorthogonal, ri, ci, pe, left, right, np))
    k = Int(np[])
    return (rowindices=ri[1:k], colindices=ci[1:k], pivoterrors=pe[1:k+1], left=left[:, 1:k],
            right=reshape(right[1:k*n], k, n))
end

# ------------------------------------------------------------------ device buffers (AMDGPU.jl ROCArray pointers)
# rrlu(A) of a device matrix with the copy (matrixlu.jl:462) fused into the first pass: dA untouched,
# dW (even ld, 16-byte aligned, not overlapping) the work matrix
function device_rrlu_copy!(ctx::Ctx, dA::Ptr{Float64}, lda::Integer, dW::Ptr{Float64}, m::Integer, n::Integer,
        ldw::Integer; maxrank::Int=typemax(Int), reltol::Float64=1e-14, abstol::Float64=0.0, leftorthogonal::Bool=true)
    rp = Vector{Int64}(undef, m); cp = Vector{Int64}(undef, n)
    np = Ref{Int64}(0); err = Ref{Float64}(0.0); pe = Vector{Float64}(undef, min(maxrank, m, n) + 1)
    check(ctx, ccall((:tci_rrlu_copy_d, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64, Int64, Int64, Float64, Float64,
         Cint, Ptr{Int64}, Ptr{Int64}, Ref{Int64}, Ref{Float64}, Ptr{Float64}),
        ctx.h, dA, lda, dW, m, n, ldw, maxrank, reltol, abstol, leftorthogonal, rp, cp, np, err, pe))
    return rp, cp, Int(np[]), err[], pe
end

# the blocked Schur update C -= W * V on fp64 MFMA, as mul!(C, W, V, -1.0, 1.0)
schur_update!(ctx::Ctx, dC::Ptr{Float64}, m, n, ldc, dW::Ptr{Float64}, ldw, dV::Ptr{Float64}, ldv, k) =
    check(ctx, ccall((:tci_schur_update_d, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
        ctx.h, dC, m, n, ldc, dW, ldw, dV, ldv, k))

# a block of Pi evaluated into device memory with host index tables (asynchronous upload, max|Pi|
# folded into the device word maxbits, no host synchronisation)
batcheval_async!(f::GPUBatchEvaluator, Itab::Vector{Int32}, m, nl, Jtab::Vector{Int32}, n, nr,
                 dPi::Ptr{Float64}, ldpi, maxbits::Ptr{UInt64}) =
    check(f.ctx, ccall((:tci_batcheval_da, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Int32}, Int64, Int32, Ptr{Int32}, Int64, Int32, Int32,
         Ptr{Float64}, Int64, Ptr{UInt64}),
        f.ctx.h, f.h, Itab, m, nl, Jtab, n, nr, 0, dPi, ldpi, maxbits))

# ------------------------------------------------------------------ multi-GPU (one process per GPU)
mutable struct GPUComm
    h::Ptr{Cvoid}
    nranks::Int
    rank::Int
end

# rank 0 creates the 128-byte id; the caller broadcasts it (MPI.Bcast! / a RemoteChannel)
function unique_id()
    id = Vector{UInt8}(undef, 128)
    nb = Ref{Int64}(0)
    st = ccall((:tci_comm_unique_id, libtci), Cint, (Ptr{UInt8}, Ref{Int64}), id, nb)
    st == TCI_OK || error("tci_comm_unique_id failed ($st)")
    return id[1:nb[]]
end

function GPUComm(ctx::Ctx, nranks::Integer, rank::Integer, id::Vector{UInt8})
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ctx, ccall((:tci_comm_create, libtci), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}, Ref{Ptr{Cvoid}}),
                     ctx.h, nranks, rank, id, r))
    c = GPUComm(r[], nranks, rank)
    finalizer(c) do c
        c.h == C_NULL || ccall((:tci_comm_destroy, libtci), Cint, (Ptr{Cvoid},), c.h)
        c.h = C_NULL
    end
    return c
end

# The column-sharded rrLU: this rank holds columns c0:c0+nloc-1 (0-based c0) of the m x n Pi at dA
# (ld lda, plus one scratch column); every rank gets the same pivots, bitwise the single-GPU ones
function rrlu_sharded(ctx::Ctx, comm::GPUComm, dA::Ptr{Float64}, m, nloc, lda, c0, n; maxrank::Int=typemax(Int),
        reltol::Float64=1e-14, abstol::Float64=0.0, leftorthogonal::Bool=true)
    rowperm = Vector{Int64}(undef, m); colperm = Vector{Int64}(undef, n)
    np = Ref{Int64}(0); err = Ref{Float64}(0.0); pe = Vector{Float64}(undef, min(maxrank, m, n) + 1)
    check(ctx, ccall((:tci_rrlu_sharded_d, libtci), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Float64}, Int64, Int64, Int64,
         Int64, Int64, Int64, Float64, Float64, Cint, Ptr{Int64}, Ptr{Int64}, Ref{Int64},
         Ref{Float64}, Ptr{Float64}),
        ctx.h, comm.h, C_NULL, C_NULL, comm.nranks, dA, m, nloc, lda, c0, n, maxrank, reltol, abstol,
        leftorthogonal, rowperm, colperm, np, err, pe))
    k = Int(np[])
    return rowperm[1:k], colperm[1:k], k, err[], pe[1:k+1]
end

# L (m x np, replicated) and this rank's columns of U (np x n) of the last rrlu_sharded on ctx
function rrlu_sharded_factors(ctx::Ctx, m, n, np)
    L = Matrix{Float64}(undef, m, max(np, 1)); U = zeros(Float64, max(np, 1), n)
    check(ctx, ccall((:tci_rrlu_sharded_factors_h, libtci), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64),
                     ctx.h, L, U, max(np, 1)))
    return L[:, 1:np], U[1:np, :]
end

end # module
