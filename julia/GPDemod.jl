# GPDemod.jl — the Julia side of the drop-in boundary (include/gpdemod.h).
#
# A maintainer `include`s this file inside `module GPPupilDemodulation` (after Modulation.jl and
# Faint.jl), so that `idx`, `FT`/`SC`/`FC`, `M_2PI`, `MetState`, `FaintStates`,
# `ModulationNoOffsets`/`ModulationWithOffsets` resolve to the reference's own definitions
# (src/Modulation.jl:9-55, src/Faint.jl:1-19).  `demodulateall_gpu` keeps the signature, keywords
# and return value of `demodulateall` (src/Modulation.jl:344-351, 434); the diode loop
# (src/Modulation.jl:387-433) becomes one `ccall`.  The calling convention mirrors the reference's
# only native call, `ccall((:ffcrimll, libcfitsio), …)` + `fits_assert_ok` (src/FitsUtils.jl:40-59):
# integer status, 0 = ok, message in a caller-owned buffer.
#
# Every `ccall` argument tuple below is checked against include/gpdemod.h, argument by argument,
# by tests/test_julia_shim.py (Julia is not installed in the build container).

const libgpdemod = get(ENV, "GPDEMOD_LIB",
                       joinpath(@__DIR__, "..", "gppupildemodulation.jl_amd", "libgpdemod.so"))

"""include/gpdemod.h `gpd_param` (64 bytes): the Modulation record plus the likelihood."""
struct GpdParam
    c::ComplexF64
    a::ComplexF64
    b::Float64
    ϕ::Float64
    chi2::Float64
    nfev::Int32
    status::Int32
end

const GPD_FIT_OFFSETS = 0x1
const GPD_RECENTER = 0x2
const GPD_ONLY_HIGH = 0x4
const GPD_METHOD_EXACT = 0x10
const GPD_METHOD_HARMONIC = 0x20

const GPD_ST_REFIT = 0x1
const GPD_ST_MAXFUN = 0x2
const GPD_ST_NAN = 0x4
const GPD_ST_EXACT = 0x8
const GPD_ST_FALLBACK = 0x10
const GPD_ST_SYNC = 0x20

"""Throw on a negative status, with the library's message (as `fits_assert_ok`)."""
function gpd_assert_ok(rc::Integer, err::Vector{UInt8})
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:gpd_strerror, libgpdemod), Cstring, (Cint,), rc))
    n = something(findfirst(==(0x00), err), length(err) + 1) - 1
    error("gpdemod error $rc ($msg): " * String(err[1:n]))
end

gpd_version() = ccall((:gpd_version, libgpdemod), Cint, ())
gpd_device_count() = ccall((:gpd_device_count, libgpdemod), Cint, ())
# id of the sources the loaded library was built from (build.py's tree id; provenance checks)
gpd_build_id() = unsafe_string(ccall((:gpd_build_id, libgpdemod), Cstring, ()))
gpd_release(device::Integer=0) = ccall((:gpd_release, libgpdemod), Cint, (Cint,), device)

method_flags(method::Symbol) =
    method === :auto ? 0x0 : method === :exact ? GPD_METHOD_EXACT :
    method === :harmonic ? GPD_METHOD_HARMONIC : error("method must be :auto, :exact or :harmonic")

# 0-based FC column of diode column c (1..32) in the 40-column idx() layout (src/Modulation.jl:388)
fc_columns() = Int32[idx(c <= 16 ? FT : SC, (c - 1) % 16 ÷ 4 + 1, FC) - 1 for c in 1:32]

"""buildstates (src/Faint.jl:21-73) in the library (host).  `timer1`/`timer2` already shifted by
lag·Δt, as FaintStates holds them."""
function gpd_buildstates(t::AbstractVector, timer1::AbstractVector, timer2::AbstractVector;
                         preswitchdelay=0.01, postwitchdelay=0.3)
    tt = Vector{Float64}(t)
    t1 = Vector{Float64}(timer1)
    t2 = Vector{Float64}(timer2)
    st = Vector{Int8}(undef, length(tt))
    rc = ccall((:gpd_buildstates, libgpdemod), Cint,
               (Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Float64, Float64,
                Ptr{Int8}),
               length(tt), tt, length(t1), t1, length(t2), t2, preswitchdelay, postwitchdelay, st)
    rc == 0 || error("gpd_buildstates failed: $rc")
    return st
end

function faint_state_vector(faintparam, t, preswitchdelay, postwitchdelay)
    faintparam === nothing && return C_NULL
    faintparam isa FaintStates &&
        return gpd_buildstates(t, faintparam.timer1, faintparam.timer2;
                               preswitchdelay=preswitchdelay, postwitchdelay=postwitchdelay)
    return Int8.(Integer.(faintparam))  # AbstractVector{MetState}
end

"""
    demodulateall_gpu(timestamp, data; init=:auto, recenter=true, faintparam=nothing,
                      onlyhigh=false, fitoffsets=false, preswitchdelay=0.01,
                      postwitchdelay=0.3, method=:auto, n_gpus=1)

GPU drop-in for `demodulateall` (src/Modulation.jl:344-435): same arguments, same
`(output, param, likelihood)`.  `data` is N×40 in idx() order (32 diodes, 8 FC columns).
A `Matrix{ComplexF32}` stays Float32 in device memory (`gpd_fit_batch_c32`, Float64 arithmetic).
"""
function demodulateall_gpu(timestamp::AbstractVector, data::AbstractMatrix{Complex{T}};
                           init::Union{Symbol,AbstractVector}=:auto, recenter::Bool=true,
                           faintparam=nothing, onlyhigh::Bool=false, fitoffsets::Bool=false,
                           preswitchdelay=0.01, postwitchdelay=0.3, method::Symbol=:auto,
                           n_gpus::Integer=1) where {T<:AbstractFloat}
    N = size(data, 1)
    size(data, 2) == 40 || error("data must be N×40 (32 diodes + 8 FC columns)")
    length(timestamp) == N || error("voltage and time must have the same number of lines")
    t = Vector{Float64}(timestamp)
    c32 = T === Float32
    # the exposure as it is (no conversion copy when it already is a Matrix of the library's
    # element type); ComplexF32 stays Float32 in device memory
    d = c32 ? (data isa Matrix{ComplexF32} ? data : Matrix{ComplexF32}(data)) :
              (data isa Matrix{ComplexF64} ? data : Matrix{ComplexF64}(data))
    state = faint_state_vector(faintparam, t, preswitchdelay, postwitchdelay)
    flags = UInt32((recenter ? GPD_RECENTER : 0) | (fitoffsets ? GPD_FIT_OFFSETS : 0) |
                   (onlyhigh ? GPD_ONLY_HIGH : 0) | method_flags(method))
    xinit = init isa Symbol ? C_NULL : Vector{Float64}(init)
    params = Vector{GpdParam}(undef, 32)
    # the reference's `output = copy(data)` then the diode loop (src/Modulation.jl:353,
    # 417-425): one call fills a fresh matrix — the 32 demodulated diodes and the FC columns
    # 33..40 as given — so the exposure is never copied on this side; ComplexF32 data gets a
    # ComplexF32 output (Complex{T}.(…) of the Float64 results)
    output = similar(d)
    err = zeros(UInt8, 512)
    GC.@preserve t d state xinit params output err begin
        if c32
            rc = ccall((:gpd_demodulateall_c32, libgpdemod), Cint,
                       (Int64, Ptr{Float64}, Ptr{ComplexF32}, Int64, Ptr{Int8}, Ptr{Float64},
                        UInt32, Int32, Ptr{GpdParam}, Ptr{ComplexF32}, Int64, Int32, Ptr{UInt8},
                        Csize_t),
                       N, t, d, N, state, xinit, flags, 60, params, output, N, n_gpus, err,
                       length(err))
        else
            rc = ccall((:gpd_demodulateall, libgpdemod), Cint,
                       (Int64, Ptr{Float64}, Ptr{ComplexF64}, Int64, Ptr{Int8}, Ptr{Float64},
                        UInt32, Int32, Ptr{GpdParam}, Ptr{ComplexF64}, Int64, Int32, Ptr{UInt8},
                        Csize_t),
                       N, t, d, N, state, xinit, flags, 60, params, output, N, n_gpus, err,
                       length(err))
        end
        gpd_assert_ok(rc, err)
    end
    # the reference's return types (src/Modulation.jl:353-359, 434): output::Matrix{Complex{T}},
    # param::Vector{Modulation…{T}}, likelihood::Vector{T}; the library's Float64 records are
    # converted to T
    param = fitoffsets ?
        ModulationWithOffsets{T}[ModulationWithOffsets{T}(p.c, p.a, p.b, p.ϕ, M_2PI) for p in params] :
        ModulationNoOffsets{T}[ModulationNoOffsets{T}(p.a, p.b, p.ϕ, M_2PI) for p in params]
    likelihood = T[p.chi2 for p in params]
    # eltype(output) == eltype(data) for every T (advisor r5): Float32/Float64 data came back in
    # its own type; any other T (Float16, BigFloat, …) went through ComplexF64, so it gets the
    # reference's `output = copy(data)` with the 32 demodulated columns converted into it — the
    # FC columns 33..40 keep their own precision
    if !(T === Float32 || T === Float64)
        out = copy(data)
        out[:, 1:32] .= Complex{T}.(view(output, :, 1:32))
        output = out
    end
    return (output, param, likelihood)
end

"""χ²(b, ϕ) of the 32 diodes at caller-given points (the `lkl` functor, src/Modulation.jl:318-330)."""
function chi2_gpu(timestamp::AbstractVector, data::AbstractMatrix{Complex{T}}, bphi::AbstractMatrix;
                  faintparam=nothing, onlyhigh::Bool=false, fitoffsets::Bool=false,
                  preswitchdelay=0.01, postwitchdelay=0.3, method::Symbol=:auto,
                  n_gpus::Integer=1) where {T<:AbstractFloat}
    N = size(data, 1)
    t = Vector{Float64}(timestamp)
    d = Matrix{ComplexF64}(data)
    bp = Matrix{Float64}(bphi)          # 2×32: (b, ϕ) per diode
    size(bp) == (2, 32) || error("bphi must be 2×32")
    state = faint_state_vector(faintparam, t, preswitchdelay, postwitchdelay)
    fcop = fc_columns()
    flags = UInt32((fitoffsets ? GPD_FIT_OFFSETS : 0) | (onlyhigh ? GPD_ONLY_HIGH : 0) |
                   method_flags(method))
    params = Vector{GpdParam}(undef, 32)
    err = zeros(UInt8, 512)
    GC.@preserve t d state bp params err begin
        rc = ccall((:gpd_chi2_batch, libgpdemod), Cint,
                   (Int64, Int64, Ptr{Float64}, Ptr{ComplexF64}, Int64, Ptr{ComplexF64}, Int64,
                    Int64, Ptr{Int32}, Ptr{Int8}, Float64, Ptr{Float64}, UInt32, Ptr{GpdParam},
                    Int32, Ptr{UInt8}, Csize_t),
                   N, 32, t, d, N, d, 40, N, fcop, state, M_2PI, bp, flags, params, n_gpus,
                   err, length(err))
        gpd_assert_ok(rc, err)
    end
    return T[p.chi2 for p in params]    # lkl returns T (src/Modulation.jl:318-326)
end

"""
    demodulate_windows_gpu(times, cmplxV, nwindow; …) -> (output, params)

processmetrology's windowed mode (src/GPPupilDemodulation.jl:191-225): every window of `nwindow`
samples (Iterators.partition, the last one shorter) fitted as its own demodulateall call, all
windows × diodes in one call.  `params[32w + k]` = diode k of window w (window-major).
"""
function demodulate_windows_gpu(times::AbstractVector, cmplxV::AbstractMatrix{<:Complex},
                                nwindow::Integer; recenter::Bool=true, faintparam=nothing,
                                onlyhigh::Bool=false, fitoffsets::Bool=false,
                                preswitchdelay=0.01, postwitchdelay=0.3, method::Symbol=:auto,
                                n_gpus::Integer=1)
    N = size(cmplxV, 1)
    t = Vector{Float64}(times)
    d = Matrix{ComplexF64}(cmplxV)
    state = faint_state_vector(faintparam, t, preswitchdelay, postwitchdelay)
    fcop = fc_columns()
    flags = UInt32((recenter ? GPD_RECENTER : 0) | (fitoffsets ? GPD_FIT_OFFSETS : 0) |
                   (onlyhigh ? GPD_ONLY_HIGH : 0) | method_flags(method))
    nwin = cld(N, nwindow)
    params = Vector{GpdParam}(undef, 32 * nwin)
    output = copy(d)
    err = zeros(UInt8, 512)
    GC.@preserve t d state params output err begin
        rc = ccall((:gpd_fit_windows, libgpdemod), Cint,
                   (Int64, Int64, Int64, Ptr{Float64}, Ptr{ComplexF64}, Int64, Ptr{ComplexF64},
                    Int64, Int64, Ptr{Int32}, Ptr{Int8}, Float64, Ptr{Float64}, UInt32, Int32,
                    Ptr{GpdParam}, Ptr{ComplexF64}, Int64, Int32, Ptr{UInt8}, Csize_t),
                   N, nwindow, 32, t, d, N, d, 40, N, fcop, state, M_2PI, C_NULL, flags, 60,
                   params, output, N, n_gpus, err, length(err))
        gpd_assert_ok(rc, err)
    end
    return (output, params)
end

"""
    process_volt_gpu(times, volt, offsets; window=0, state=C_NULL, fitoffsets=false)

processmetrology's numeric core straight from the FITS VOLT column (src/GPPupilDemodulation.jl:
147-171, 191-207): `volt` is the 80×N Float32 matrix FITSIO returns; `offsets` the 40 centres
(or `nothing`).  Returns (demodulated VOLT, Float32 80×N; params).
"""
function process_volt_gpu(times::AbstractVector, volt::Matrix{Float32}, offsets;
                          window::Integer=0, state=C_NULL, recenter::Bool=true,
                          fitoffsets::Bool=false, device::Integer=0)
    N = size(volt, 2)
    size(volt, 1) == 80 || error("VOLT must be 80×N")
    t = Vector{Float64}(times)
    cen = offsets === nothing ? C_NULL : Vector{ComplexF64}(offsets)
    flags = UInt32((recenter ? GPD_RECENTER : 0) | (fitoffsets ? GPD_FIT_OFFSETS : 0))
    params = Vector{GpdParam}(undef, window == 0 ? 32 : 32 * cld(N, window))
    out = similar(volt)
    err = zeros(UInt8, 512)
    GC.@preserve t volt cen state params out err begin
        rc = ccall((:gpd_process_volt, libgpdemod), Cint,
                   (Int64, Ptr{Float64}, Ptr{Float32}, Int64, Ptr{ComplexF64}, Ptr{Int8}, Float64,
                    Ptr{Float64}, UInt32, Int32, Int64, Ptr{GpdParam}, Ptr{Float32}, Int64, Cint,
                    Ptr{UInt8}, Csize_t),
                   N, t, volt, 80, cen, state, M_2PI, C_NULL, flags, 60, window, params, out, 80,
                   device, err, length(err))
        gpd_assert_ok(rc, err)
    end
    return (out, params)
end
