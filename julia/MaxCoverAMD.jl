#=
MaxCoverAMD.jl — Julia binding of libmaxcover (include/maxcover.h) for the reference
Gabisanth/MaximumAreaCoverageOptimization.jl. Drop-in replacements for the hot path:

  calculateArea(circles, points)            src/AreaCoverageCalculation.jl:63-110
  createObjective(cells, N, r_max)          src/TDM_STATIC_opt.jl:82-100
  rmvCoveredPOI(cells, circles)             src/CellFunctions.jl:81-108
  poll_best(...)                            DirectSearch's poll step, src/TDM_STATIC_opt.jl:162

Plain `ccall` over the C ABI: no Julia package dependencies. The library path comes from
ENV["MAXCOVER_LIB"] or defaults to the in-tree build. Not executed in this repository's CI
(Julia is not installed in the build image); the ctypes mirror
(maximumareacoverageoptimization.jl_amd/_lib.py) makes the same calls with the same arrays and
is what the parity tests exercise. See INTEGRATION.md.
=#
module MaxCoverAMD

export MacContext, set_points!, calculateArea, createObjective, objective_batch, poll_best,
       poll_basis, rmvCoveredPOI!, area_batch, mads_run

const libmaxcover = get(ENV, "MAXCOVER_LIB",
    joinpath(@__DIR__, "..", "maximumareacoverageoptimization.jl_amd", "libmaxcover.so"))

const MAC_OK = Int32(0)
const MAC_E_SIZE = Int32(2)

struct MaxCoverError <: Exception
    code::Int32
    msg::String
end
Base.showerror(io::IO, e::MaxCoverError) = print(io, "libmaxcover error ", e.code, ": ", e.msg)

function check(rc::Int32)
    rc == MAC_OK && return nothing
    msg = unsafe_string(ccall((:mac_last_error, libmaxcover), Cstring, ()))
    # the reference's own error for a length that is not a multiple of 3 (Int(length/3))
    rc == MAC_E_SIZE && throw(InexactError(:Int, Int, msg))
    throw(MaxCoverError(rc, msg))
end

"""One device context (one GPU); the point list lives in its HBM between MADS calls."""
mutable struct MacContext
    ptr::Ptr{Cvoid}
    function MacContext(device::Integer = 0)
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:mac_ctx_create, libmaxcover), Int32, (Ref{Ptr{Cvoid}}, Int32), out, device))
        ctx = new(out[])
        finalizer(c -> ccall((:mac_ctx_destroy, libmaxcover), Cvoid, (Ptr{Cvoid},), c.ptr), ctx)
        return ctx
    end
end
Base.unsafe_convert(::Type{Ptr{Cvoid}}, c::MacContext) = c.ptr

const _default = Ref{Union{Nothing,MacContext}}(nothing)
default_context() = (_default[] === nothing && (_default[] = MacContext(0)); _default[])

# Vector{Vector{Float64}} records [x, y, area, importance, covered] -> contiguous 5 x M
function pack_records(points::AbstractVector{<:AbstractVector{Float64}})
    M = length(points)
    rec = Matrix{Float64}(undef, 5, M)
    @inbounds for p in 1:M
        r = points[p]
        for j in 1:5
            rec[j, p] = r[j]
        end
    end
    return rec
end

"""Upload the point list (once per MPC step, after the list changes)."""
function set_points!(ctx::MacContext, points::AbstractVector{<:AbstractVector{Float64}})
    rec = pack_records(points)
    check(ccall((:mac_set_points_records_f64, libmaxcover), Int32,
                (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64), ctx, rec, size(rec, 2), 5))
    return ctx
end

"""calculateArea(circles, points) — src/AreaCoverageCalculation.jl:63-110 (uploads points)."""
function calculateArea(circles::Vector{Float64}, points::AbstractVector{<:AbstractVector{Float64}};
                       ctx::MacContext = default_context())
    set_points!(ctx, points)
    return calculateArea(circles, ctx)
end

"""calculateArea against the context's resident point list."""
function calculateArea(circles::Vector{Float64}, ctx::MacContext)
    out = Ref{Float64}(0.0)
    check(ccall((:mac_area_f64, libmaxcover), Int32,
                (Ptr{Cvoid}, Ptr{Float64}, Int64, Ref{Float64}), ctx, circles, length(circles), out))
    return out[]
end

"""K candidates as the columns of a 3N x K matrix."""
function area_batch(cands::Matrix{Float64}, ctx::MacContext)
    out = Vector{Float64}(undef, size(cands, 2))
    check(ccall((:mac_area_batch_f64, libmaxcover), Int32,
                (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Ptr{Float64}),
                ctx, cands, size(cands, 1), size(cands, 2), out))
    return out
end

function objective_batch(cands::Matrix{Float64}, r_max::Vector{Float64}, ctx::MacContext;
                         penalty::Float64 = 1e5)
    out = Vector{Float64}(undef, size(cands, 2))
    check(ccall((:mac_objective_batch_f64, libmaxcover), Int32,
                (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Ptr{Float64}, Float64, Ptr{Float64}),
                ctx, cands, size(cands, 1), size(cands, 2), r_max, penalty, out))
    return out
end

"""
createObjective(cells, N, r_max) — drop-in for src/TDM_STATIC_opt.jl:82-100.

Uploads `cells.points_of_interest` once (the reference rebuilds the closure every MPC step,
src/FullSimulation.jl:84,95, right after the list changes) and returns the same closure
signature `x::Vector{Float64} -> Float64`: -area + 1e5 * sum |x[2N+i] - r_max[i]|, the penalty
accumulated sequentially on the host exactly as :89-97. `r_max` is captured by reference
(it is mutated between steps, src/FullSimulation.jl:64-76).
"""
function createObjective(cells, N::Integer, r_max::AbstractVector{Float64};
                         ctx::MacContext = default_context())
    set_points!(ctx, cells.points_of_interest)
    function AreaMaxObjective(x::Vector{Float64})
        area = calculateArea(x, ctx)
        violation = 0.0
        for i in 1:N
            violation += abs(x[i + 2N] - r_max[i])
        end
        return -area + violation * 1e5
    end
    return AreaMaxObjective
end

"""
poll_best(cands, r_max; prev, d_lim, tan_half_fov) — one whole MADS poll on the GPU: every
candidate's objective, cons3 (src/TDM_Constraints.jl:54-75) as an extreme barrier (+Inf), and
the lowest-index minimiser. Returns (best_obj, best_idx (1-based, 0 if none feasible), objs).
"""
function poll_best(cands::Matrix{Float64}, r_max::Vector{Float64}, ctx::MacContext;
                   penalty::Float64 = 1e5, prev::Union{Nothing,Vector{Float64}} = nothing,
                   d_lim::Union{Nothing,Vector{Float64}} = nothing, tan_half_fov::Float64 = 1.0)
    K = size(cands, 2)
    objs = Vector{Float64}(undef, K)
    bo = Ref{Float64}(Inf)
    bi = Ref{Int64}(-1)
    pprev = prev === nothing ? Ptr{Float64}(C_NULL) : pointer(prev)
    pdlim = d_lim === nothing ? Ptr{Float64}(C_NULL) : pointer(d_lim)
    GC.@preserve prev d_lim begin
        check(ccall((:mac_poll_best_f64, libmaxcover), Int32,
                    (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Ptr{Float64}, Float64,
                     Ptr{Float64}, Ptr{Float64}, Float64, Ptr{Float64}, Ref{Float64}, Ref{Int64}),
                    ctx, cands, size(cands, 1), K, r_max, penalty, pprev, pdlim, tan_half_fov,
                    objs, bo, bi))
    end
    return bo[], bi[] + 1, objs
end

"""
poll_basis(x_inc, L, rp, cp, delta, r_max, ctx; prev, d_lim, tan_half_fov) — a DirectSearch-owned
poll in basis form (src/TDM_STATIC_opt.jl:22-44 CustomPoll's b / i / maximal_basis; :162): the 2n
candidates x_inc ± delta * B[:, k], B = L[rp, cp] (L lower triangular, rp / cp permutations,
1-based here as in Julia), expanded on the GPU — 2.4 MB shipped at n = 1536 instead of the 37.7-MB
matrix. Returns (best_obj, best_idx (1-based over [plus directions; minus directions], 0 if none
feasible), objs).
"""
function poll_basis(x_inc::Vector{Float64}, L::AbstractMatrix{<:Integer}, rp::AbstractVector{<:Integer},
                    cp::AbstractVector{<:Integer}, delta::Float64, r_max::Vector{Float64},
                    ctx::MacContext; penalty::Float64 = 1e5,
                    prev::Union{Nothing,Vector{Float64}} = nothing,
                    d_lim::Union{Nothing,Vector{Float64}} = nothing, tan_half_fov::Float64 = 1.0)
    n = length(x_inc)
    tri = Vector{Int16}(undef, n * (n + 1) ÷ 2)
    q = 1
    @inbounds for r in 1:n, c in 1:r      # lower triangle packed by rows
        tri[q] = Int16(L[r, c])
        q += 1
    end
    rp0 = Int32.(rp .- 1)
    cp0 = Int32.(cp .- 1)
    objs = Vector{Float64}(undef, 2n)
    bo = Ref{Float64}(Inf)
    bi = Ref{Int64}(-1)
    pprev = prev === nothing ? Ptr{Float64}(C_NULL) : pointer(prev)
    pdlim = d_lim === nothing ? Ptr{Float64}(C_NULL) : pointer(d_lim)
    GC.@preserve prev d_lim begin
        check(ccall((:mac_poll_basis_f64, libmaxcover), Int32,
                    (Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Int16}, Ptr{Int32}, Ptr{Int32}, Float64,
                     Ptr{Float64}, Float64, Ptr{Float64}, Ptr{Float64}, Float64, Ptr{Float64},
                     Ref{Float64}, Ref{Int64}),
                    ctx, x_inc, n, tri, rp0, cp0, delta, r_max, penalty, pprev, pdlim, tan_half_fov,
                    objs, bo, bi))
    end
    return bo[], bi[] + 1, objs
end

struct MadsParams
    n_iter::Int64
    ell0::Int32
    ell_max::Int32
    seed::UInt64
end
struct MadsStats
    f::Float64
    iterations::Int64
    evaluations::Int64
    status::Int32
    feasible::Int32
    seconds::Float64
    host_enqueue_s::Float64
    host_perm_s::Float64
    wait_s::Float64
    host_post_s::Float64
    feasible_evaluations::Int64
    rejected_polls::Int64
    successes::Int64
    slot_fallbacks::Int64
end

"""
mads_run(x0, r_max, ctx; prev, d_lim, tan_half_fov, n_iter, ell0, ell_max, seed) — the whole
granular-MADS loop inside libmaxcover (complete LTMADS poll generated on the device, cons3 as
extreme barrier): the batched stand-in for TDM_STATIC_opt.optimize (src/TDM_STATIC_opt.jl:118-169).
Returns (x, stats::MadsStats).
"""
function mads_run(x0::Vector{Float64}, r_max::Vector{Float64}, ctx::MacContext;
                  penalty::Float64 = 1e5, prev::Union{Nothing,Vector{Float64}} = nothing,
                  d_lim::Union{Nothing,Vector{Float64}} = nothing, tan_half_fov::Float64 = 1.0,
                  n_iter::Integer = 100, ell0::Integer = 2, ell_max::Integer = 6,
                  seed::Integer = 20250216)
    x = similar(x0)
    prm = Ref(MadsParams(n_iter, ell0, ell_max, UInt64(seed)))
    st = Ref{MadsStats}()
    pprev = prev === nothing ? Ptr{Float64}(C_NULL) : pointer(prev)
    pdlim = d_lim === nothing ? Ptr{Float64}(C_NULL) : pointer(d_lim)
    GC.@preserve prev d_lim begin
        check(ccall((:mac_mads_run, libmaxcover), Int32,
                    (Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Float64}, Float64, Ptr{Float64},
                     Ptr{Float64}, Float64, Ref{MadsParams}, Ptr{Float64}, Ref{MadsStats}),
                    ctx, x0, length(x0), r_max, penalty, pprev, pdlim, tan_half_fov, prm, x, st))
    end
    return x, st[]
end

"""
rmvCoveredPOI!(cells, circles) — src/CellFunctions.jl:81-108: delete, order-preserving, every
entry of cells.points_of_interest covered by `circles`; the device list is updated in place.
"""
function rmvCoveredPOI!(cells, circles::Vector{Float64}; ctx::MacContext = default_context())
    pts = cells.points_of_interest
    set_points!(ctx, pts)
    kept = Vector{Int64}(undef, length(pts))
    M = Ref{Int64}(0)
    check(ccall((:mac_remove_covered_f64, libmaxcover), Int32,
                (Ptr{Cvoid}, Ptr{Float64}, Int64, Ptr{Int64}, Ref{Int64}),
                ctx, circles, length(circles), kept, M))
    cells.points_of_interest = pts[kept[1:M[]] .+ 1]
    return cells
end

end # module
