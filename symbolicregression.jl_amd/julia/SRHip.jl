# SRHip.jl — the Julia side of the drop-in boundary (ccall into libsrhip.so).
#
# This is the binding a SymbolicRegression.jl maintainer would add (INTEGRATION.md
# shows where it plugs in). UNTESTED AS JULIA: the build image has no Julia, so
# this file has never been executed. What is tested (tests/test_julia_binding.py,
# CPU): every `ccall((:srhip_*, libsrhip), R, (A...), ...)` below names a symbol
# that include/srhip.h declares and libsrhip.so exports, with the declared number
# of arguments and compatible argument / return types; and every loss type maps
# to a SRHIP_LOSS_* code. The C ABI itself is exercised from Python through the
# same entry points (tests/test_abi.py, tests/test_gpu_parity.py, ...).
module SRHip

using DynamicExpressions: Node, count_nodes, set_constants
using LossFunctions: L2DistLoss, L1DistLoss, LPDistLoss, HuberLoss, LogCoshLoss, L1EpsilonInsLoss,
    L2EpsilonInsLoss, QuantileLoss, PeriodicLoss, LogitDistLoss
import ..CoreModule: Options, Dataset

const libsrhip = get(ENV, "SRHIP_LIB", joinpath(@__DIR__, "..", "lib", "libsrhip.so"))

# include/srhip.h
const SRHIP_OK = Int32(0)
const SRHIP_ERR_UNSUPPORTED = Int32(-2)
const NODE_CONST, NODE_FEATURE, NODE_UNARY, NODE_BINARY = UInt8(0), UInt8(1), UInt8(2), UInt8(3)
const X_JULIA = Int32(0)
const LOSS_L2, LOSS_L1, LOSS_LP, LOSS_HUBER, LOSS_LOGCOSH = Int32(0), Int32(1), Int32(2), Int32(3), Int32(4)
const LOSS_L1EPSINS, LOSS_L2EPSINS, LOSS_QUANTILE, LOSS_PERIODIC, LOSS_LOGITDIST, LOSS_LPINT =
    Int32(5), Int32(6), Int32(7), Int32(8), Int32(9), Int32(10)

struct SrhipTrees              # include/srhip.h: srhip_trees
    ntrees::Int32
    node_off::Ptr{Int32}
    kind::Ptr{UInt8}
    arg::Ptr{UInt16}
    const_off::Ptr{Int32}
    consts::Ptr{Cvoid}
end

"""Raised for anything outside the engine's coverage: the caller falls back to
the reference CPU path (srhip.h: SRHIP_ERR_UNSUPPORTED)."""
struct Unsupported <: Exception
    msg::String
end

last_error() = unsafe_string(ccall((:srhip_last_error, libsrhip), Cstring, ()))
const SRHIP_ERR_INVALID = Int32(-1)
function check(rc::Int32)
    rc == SRHIP_OK && return nothing
    rc == SRHIP_ERR_UNSUPPORTED && throw(Unsupported(last_error()))
    # malformed input, e.g. a program and a dataset on different devices
    rc == SRHIP_ERR_INVALID && throw(ArgumentError("srhip: $(last_error())"))
    error("srhip: $(last_error())")
end

dtype_code(::Type{Float32}) = Int32(0)
dtype_code(::Type{Float64}) = Int32(1)
dtype_code(::Type) = throw(Unsupported("only Float32/Float64 run on the GPU"))

# ---- elementwise losses -> SRHIP_LOSS_* (LossFunctions.jl distance losses,
# src/Options.jl:429-431 default L2DistLoss; docs/src/losses.md) ----------------
loss_code(::L2DistLoss) = (LOSS_L2, 0.0)
loss_code(::L1DistLoss) = (LOSS_L1, 0.0)
# LPDistLoss{P} with an Int P keeps Julia's T^Integer rules (srhip.h SRHIP_LOSS_LPINT)
loss_code(::LPDistLoss{P}) where {P} = (P isa Integer ? LOSS_LPINT : LOSS_LP, Float64(P))
loss_code(l::HuberLoss) = (LOSS_HUBER, Float64(l.d))
loss_code(::LogCoshLoss) = (LOSS_LOGCOSH, 0.0)
loss_code(l::L1EpsilonInsLoss) = (LOSS_L1EPSINS, Float64(l.ε))
loss_code(l::L2EpsilonInsLoss) = (LOSS_L2EPSINS, Float64(l.ε))
loss_code(l::QuantileLoss) = (LOSS_QUANTILE, Float64(l.τ))
# PeriodicLoss stores k = 2π/circumference; the engine takes the circumference
loss_code(l::PeriodicLoss) = (LOSS_PERIODIC, 2π / Float64(l.k))
loss_code(::LogitDistLoss) = (LOSS_LOGITDIST, 0.0)
loss_code(l) = throw(Unsupported("elementwise loss $(typeof(l)) is not in the engine's table"))

# ---- contexts: one per (thread, device); calls through a context are serialised.
# An evaluation runs on its PROGRAM's context (srhip.h): programs are created
# in the calling thread's context, datasets are uploaded once per device and
# shared by every thread's context, so threads (one island each,
# src/SearchUtils.jl:33-45) score concurrently. A task that migrates between
# threads keeps using the context its program was created in, which is safe
# (the context's mutex serialises it with that thread's calls).
const CTX = Dict{Tuple{Int,Int},Ptr{Cvoid}}()
const CTX_LOCK = ReentrantLock()
function context(device::Int=0)
    key = (Threads.threadid(), device)
    lock(CTX_LOCK) do
        get!(CTX, key) do
            h = Ref{Ptr{Cvoid}}(C_NULL)
            check(ccall((:srhip_open, libsrhip), Int32, (Int32, Ptr{Ptr{Cvoid}}), device, h))
            h[]
        end
    end
end

function device_available()
    n = Ref{Int32}(0)
    try
        ccall((:srhip_device_count, libsrhip), Int32, (Ptr{Int32},), n) == SRHIP_OK && n[] > 0
    catch
        false  # library missing or not loadable
    end
end

# ---- operator ids (srhip_op_lookup applies binopmap/unaopmap names) ------------
function op_id(op, arity)
    a = Ref{Int32}(0); i = Ref{Int32}(0)
    check(ccall((:srhip_op_lookup, libsrhip), Int32, (Cstring, Ptr{Int32}, Ptr{Int32}),
                string(nameof(op)), a, i))
    a[] == arity || throw(Unsupported("operator $(op) has arity $(a[])"))
    return UInt16(i[])
end
const OPS_CACHE = IdDict{Any,Any}()
operator_ids(options::Options) = lock(CTX_LOCK) do
    get!(OPS_CACHE, options) do
        ([op_id(op, 2) for op in options.operators.binops], [op_id(op, 1) for op in options.operators.unaops])
    end
end

"""
    enabled(options) -> Bool

Whether `options` can run on the engine: a device is visible, `loss_function`
is not set (arbitrary Julia stays on the CPU, src/LossFunctions.jl:60-67), the
elementwise loss and every operator are in the engine's table. Set
ENV["SRHIP_DISABLE"] = "1" to force the reference path.
"""
function enabled(options::Options)
    get(ENV, "SRHIP_DISABLE", "0") == "1" && return false
    # the recorder's genealogy (src/Recorder.jl, Options.jl:597-599) is written by
    # the reference's per-candidate loops: with it on, the search stays there
    options.recorder && return false
    options.loss_function === nothing || return false
    device_available() || return false
    try
        loss_code(options.elementwise_loss)
        operator_ids(options)
        return true
    catch e
        e isa Unsupported || rethrow()
        return false
    end
end

# ---- flattening: post-order node streams, constants in get_constants order ----
function flatten(trees::AbstractVector{Node{T}}, options::Options) where {T}
    bin, una = operator_ids(options)
    kind = UInt8[]; arg = UInt16[]; consts = T[]
    node_off = Int32[0]; const_off = Int32[0]
    function visit(t::Node{T})
        if t.degree == 0
            if t.constant
                push!(kind, NODE_CONST); push!(arg, 0); push!(consts, t.val::T)
            else
                push!(kind, NODE_FEATURE); push!(arg, UInt16(t.feature - 1))
            end
        elseif t.degree == 1
            visit(t.l); push!(kind, NODE_UNARY); push!(arg, una[t.op])
        else
            visit(t.l); visit(t.r); push!(kind, NODE_BINARY); push!(arg, bin[t.op])
        end
    end
    for t in trees
        visit(t)
        push!(node_off, length(kind)); push!(const_off, length(consts))
    end
    return node_off, kind, arg, const_off, consts
end

# A compiled, device-resident batch of trees (srhip_program_create); destroyed
# by the caller (`destroy`) or by the finaliser.
mutable struct Program
    h::Ptr{Cvoid}
    ntrees::Int
    const_off::Vector{Int32}
    device::Int   # its datasets are this device's (srhip.h: a call runs on the program's context)
end
function destroy(p::Program)
    p.h == C_NULL && return nothing
    ccall((:srhip_program_destroy, libsrhip), Int32, (Ptr{Cvoid},), p.h)
    p.h = C_NULL
    return nothing
end
# varying_constants: the caller will set_constants! (the candidates of
# optimize_constants), so Float32 tree code reads its constants from memory
# from the start (SRHIP_PROGRAM_VARYING_CONSTANTS: no recompile on a new set)
const PROGRAM_VARYING_CONSTANTS = UInt32(1)
function Program(trees::AbstractVector{Node{T}}, options::Options, device::Int=0;
                 varying_constants::Bool=false) where {T}
    node_off, kind, arg, const_off, consts = flatten(trees, options)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    flags = varying_constants ? PROGRAM_VARYING_CONSTANTS : UInt32(0)
    GC.@preserve node_off kind arg const_off consts begin
        tr = Ref(SrhipTrees(Int32(length(trees)), pointer(node_off), pointer(kind), pointer(arg),
                            pointer(const_off), Ptr{Cvoid}(pointer(consts))))
        check(ccall((:srhip_program_create_ex, libsrhip), Int32,
                    (Ptr{Cvoid}, Int32, Ref{SrhipTrees}, UInt32, Ptr{Ptr{Cvoid}}),
                    context(device), dtype_code(T), tr, flags, h))
    end
    p = Program(h[], length(trees), const_off, device)
    finalizer(destroy, p)
    return p
end

function set_constants!(p::Program, consts::Vector{T}) where {T}
    length(consts) == p.const_off[end] || throw(ArgumentError("expected $(p.const_off[end]) constants"))
    GC.@preserve consts check(ccall((:srhip_program_set_constants, libsrhip), Int32,
                                    (Ptr{Cvoid}, Ptr{Cvoid}), p.h, consts))
    return p
end

# ---- device datasets ----------------------------------------------------------
function upload(X::AbstractMatrix{T}, y::AbstractVector{T}, w, device::Int) where {T}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    Xc = Matrix{T}(X); yc = Vector{T}(y)
    wc = w === nothing ? nothing : Vector{T}(w)
    nfeat, n = size(Xc)
    GC.@preserve Xc yc wc begin
        check(ccall((:srhip_dataset_create, libsrhip), Int32,
                    (Ptr{Cvoid}, Int32, Int32, Ptr{T}, Ptr{T}, Ptr{T}, Int64, Int32, Int64, Int64,
                     Ptr{Ptr{Cvoid}}),
                    context(device), dtype_code(T), X_JULIA, Xc, yc,
                    wc === nothing ? Ptr{T}(C_NULL) : wc, n, nfeat, 0, n, h))
    end
    return h[]
end
destroy_dataset(h::Ptr{Cvoid}) = ccall((:srhip_dataset_destroy, libsrhip), Int32, (Ptr{Cvoid},), h)

# one device copy per (Dataset, device) (src/Dataset.jl:24-64), uploaded once
# and shared by the contexts of all threads. The table holds its Datasets
# weakly (Dataset is a mutable struct): when a Dataset is collected its entry
# goes, and the DeviceCopy's finaliser frees the device memory. Guarded by
# CTX_LOCK.
mutable struct DeviceCopy
    h::Ptr{Cvoid}
end
function free!(d::DeviceCopy)
    d.h == C_NULL && return nothing
    destroy_dataset(d.h)
    d.h = C_NULL
    return nothing
end
const DEVICE_DATASETS = WeakKeyDict{Dataset,Dict{Int,DeviceCopy}}()
function device_dataset(dataset::Dataset{T}, device::Int=0) where {T}
    lock(CTX_LOCK) do
        copies = get!(() -> Dict{Int,DeviceCopy}(), DEVICE_DATASETS, dataset)
        d = get(copies, device, nothing)
        d !== nothing && d.h != C_NULL && return d.h
        d = DeviceCopy(upload(dataset.X, dataset.y, dataset.weighted ? dataset.weights : nothing, device))
        finalizer(free!, d)
        copies[device] = d
        return d.h
    end
end
"""Free the device copies of `dataset` now (they are also freed when the
Dataset is garbage-collected)."""
function release_dataset!(dataset::Dataset)
    lock(CTX_LOCK) do
        copies = pop!(DEVICE_DATASETS, dataset, nothing)
        copies === nothing || foreach(free!, values(copies))
    end
    return nothing
end
# ---- eval_loss (src/LossFunctions.jl:34-67), batched ------------------------------
"""
    eval_loss_batch(trees, dataset, options; idx=nothing) -> Vector{T}

Batched `eval_loss` (src/LossFunctions.jl:60-67): one device launch for all
trees; T(Inf) where evaluation fails. `idx` (1-based, with repetition) is
score_func_batch's row sample (src/LossFunctions.jl:95-115).
"""
function eval_loss_batch(trees::AbstractVector{Node{T}}, dataset::Dataset{T}, options::Options;
                         idx=nothing, device::Int=0) where {T}
    node_off, kind, arg, const_off, consts = flatten(trees, options)
    nt = length(trees)
    sums = Vector{Float64}(undef, nt); ok = Vector{UInt8}(undef, nt); wsum = Ref{Float64}(0)
    kindcode, param = loss_code(options.elementwise_loss)
    params = Float64[param]
    rows = idx === nothing ? Int64[] : Int64.(idx .- 1)
    GC.@preserve node_off kind arg const_off consts sums ok params rows begin
        tr = Ref(SrhipTrees(Int32(nt), pointer(node_off), pointer(kind), pointer(arg), pointer(const_off),
                            Ptr{Cvoid}(pointer(consts))))
        # the program lives in this thread's context, the dataset is shared
        check(ccall((:srhip_eval_loss_batch_ctx, libsrhip), Int32,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Ref{SrhipTrees}, Int32, Ptr{Float64}, Ptr{Int64}, Int64, Ptr{Float64},
                     Ref{Float64}, Ptr{UInt8}),
                    context(device), device_dataset(dataset, device), tr, kindcode, params,
                    idx === nothing ? Ptr{Int64}(C_NULL) : pointer(rows), length(rows), sums, wsum, ok))
    end
    return [ok[i] == 1 ? T(sums[i] / wsum[]) : T(Inf) for i in 1:nt]
end

"""
    eval_loss_batch_rowsets(trees, dataset, options, idx::Matrix{Int}) -> Vector{T}

score_func_batch's loss (src/LossFunctions.jl:95-115) for every tree on its OWN
row sample: idx is (batch_size, ntrees), column t the 1-based rows (with
repetition) of trees[t] — one `StatsBase.sample(1:n, batch_size;
replace=true)` per candidate, as the reference draws per call (:98). One
launch (srhip_eval_loss_batch_rowsets_ctx); T(Inf) where evaluation fails.
"""
function eval_loss_batch_rowsets(trees::AbstractVector{Node{T}}, dataset::Dataset{T}, options::Options,
                                 idx::AbstractMatrix{<:Integer}; device::Int=0) where {T}
    nt = length(trees)
    size(idx, 2) == nt || throw(ArgumentError("one row sample (column of idx) per tree"))
    node_off, kind, arg, const_off, consts = flatten(trees, options)
    sums = Vector{Float64}(undef, nt); ok = Vector{UInt8}(undef, nt); wsum = Vector{Float64}(undef, nt)
    kindcode, param = loss_code(options.elementwise_loss)
    params = Float64[param]
    rows = Matrix{Int64}(idx .- 1)  # column-major: tree t's sample is contiguous ([ntrees][bs] in C)
    GC.@preserve node_off kind arg const_off consts sums ok wsum params rows begin
        tr = Ref(SrhipTrees(Int32(nt), pointer(node_off), pointer(kind), pointer(arg), pointer(const_off),
                            Ptr{Cvoid}(pointer(consts))))
        check(ccall((:srhip_eval_loss_batch_rowsets_ctx, libsrhip), Int32,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Ref{SrhipTrees}, Int32, Ptr{Float64}, Ptr{Int64}, Int64, Ptr{Float64},
                     Ptr{Float64}, Ptr{UInt8}),
                    context(device), device_dataset(dataset, device), tr, kindcode, params, rows,
                    size(rows, 1), sums, wsum, ok))
    end
    return [ok[i] == 1 ? T(sums[i] / wsum[i]) : T(Inf) for i in 1:nt]
end

"""
    eval_loss_grad_batch(p::Program, dataset, options) -> (losses, grads, ok)

Loss and ∂loss/∂c of every constant of every tree of `p` in one launch
(`srhip_eval_loss_grad`), for batched constant optimisation
(src/ConstantOptimization.jl:12-65). grads[t] is in get_constants order.
"""
function eval_loss_grad_batch(p::Program, dataset::Dataset{T}, options::Options) where {T}
    nt = p.ntrees
    ncon = Int(p.const_off[end])
    sums = Vector{Float64}(undef, nt); ok = Vector{UInt8}(undef, nt); wsum = Ref{Float64}(0)
    dloss = Vector{Float64}(undef, ncon)
    kindcode, param = loss_code(options.elementwise_loss)
    params = Float64[param]
    GC.@preserve sums ok dloss params begin
        check(ccall((:srhip_eval_loss_grad, libsrhip), Int32,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Float64},
                     Ptr{UInt8}),
                    device_dataset(dataset, p.device), p.h, kindcode, params, sums, dloss, wsum, ok))
    end
    losses = [ok[i] == 1 ? T(sums[i] / wsum[]) : T(Inf) for i in 1:nt]
    grads = [dloss[(p.const_off[i] + 1):p.const_off[i + 1]] ./ wsum[] for i in 1:nt]
    return losses, grads, ok .== 1
end

# ---- batched constant optimisation (src/ConstantOptimization.jl:22-65) ----------------
struct ConstOptOptions         # include/srhip.h: srhip_constopt_options
    algorithm::Int32
    iterations::Int32
    nrestarts::Int32
    loss_kind::Int32
    loss_params::Ptr{Float64}
    start_noise::Ptr{Float64}
    seed::UInt64
end
const OPT_BFGS, OPT_NELDERMEAD = Int32(0), Int32(1)

"""
    optimize_constants_batch!(trees, dataset, options) -> (losses, converged, num_evals)

optimize_constants (src/ConstantOptimization.jl:22-65) for every tree at once
(srhip_optimize_constants_batch): all starts of all trees in lockstep on the
engine, one launch per phase. The perturbed starts draw `randn(T, nconst)`
per restart, tree by tree, where the reference does (:47). Trees whose run
converged get the best start's constants (set_constants); the others keep
x0 (:56-63). losses[i] is the loss of trees[i] at its final constants;
num_evals[i] counts its loss evaluations (+1 for the re-score of a converged
member, :58-59).
"""
function optimize_constants_batch!(trees::AbstractVector{Node{T}}, dataset::Dataset{T}, options::Options;
                                   device::Int=0) where {T}
    algo = options.optimizer_algorithm == "BFGS" ? OPT_BFGS :
           options.optimizer_algorithm == "NelderMead" ? OPT_NELDERMEAD :
           error("Optimization function not implemented.")
    node_off, kind, arg, const_off, consts = flatten(trees, options)
    nt = length(trees)
    nr = options.optimizer_nrestarts
    noise = Float64[]
    for i in 1:nt
        nc = Int(const_off[i + 1] - const_off[i])
        nc == 0 && continue
        for _ in 1:nr
            append!(noise, Float64.(randn(T, nc)))
        end
    end
    kindcode, param = loss_code(options.elementwise_loss)
    params = Float64[param]
    out_c = similar(consts); out_l = Vector{Float64}(undef, nt)
    out_k = Vector{UInt8}(undef, nt); out_n = Vector{Float64}(undef, nt)
    GC.@preserve node_off kind arg const_off consts noise params out_c out_l out_k out_n begin
        tr = Ref(SrhipTrees(Int32(nt), pointer(node_off), pointer(kind), pointer(arg), pointer(const_off),
                            Ptr{Cvoid}(pointer(consts))))
        opts = Ref(ConstOptOptions(algo, Int32(options.optimizer_options.iterations), Int32(nr), kindcode,
                                   pointer(params), pointer(noise), UInt64(0)))
        check(ccall((:srhip_optimize_constants_batch, libsrhip), Int32,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Ref{SrhipTrees}, Ref{ConstOptOptions}, Ptr{Cvoid}, Ptr{Float64},
                     Ptr{UInt8}, Ptr{Float64}),
                    context(device), device_dataset(dataset, device), tr, opts, out_c, out_l, out_k, out_n))
    end
    converged = out_k .== 1
    for i in 1:nt
        converged[i] && set_constants(trees[i], out_c[(const_off[i] + 1):const_off[i + 1]])
    end
    return T.(out_l), converged, out_n
end

# ---- eval_tree_array (src/InterfaceDynamicExpressions.jl:50-52) -------------------
"""
    eval_tree_array(tree, X, options) -> (output, did_succeed)

Per-row outputs of one tree on the engine. X is (nfeatures, n); it is uploaded
for this call. On failure the output contents are unspecified, as in the
reference (an undef array).
"""
function eval_tree_array(tree::Node{T}, X::AbstractMatrix{T}, options::Options; device::Int=0) where {T}
    out, ok = eval_tree_array_batch([tree], X, options; device=device)
    return out[:, 1], ok[1]
end

"""
    eval_tree_array_batch(trees, X, options) -> (outputs::Matrix (n, ntrees), did_succeed::Vector{Bool})

Per-row outputs of many trees in one launch; X is uploaded for this call (it
may have changed since any earlier upload, as the reference re-reads it).
"""
function eval_tree_array_batch(trees::AbstractVector{Node{T}}, X::AbstractMatrix{T}, options::Options;
                               device::Int=0) where {T}
    n = size(X, 2)
    ds = upload(X, zeros(T, n), nothing, device)
    try
        return eval_tree_array_on(trees, ds, n, options, device)
    finally
        destroy_dataset(ds)
    end
end

"""
    eval_tree_array_batch(trees, dataset::Dataset, options) -> (outputs, did_succeed)

The same on a Dataset's X through its device copy (device_dataset, uploaded
once; a Dataset is not modified after construction). `dataset` and its
DeviceCopy are rooted across the call, so neither the WeakKeyDict entry nor
the device memory can be freed while the kernel reads it.
"""
function eval_tree_array_batch(trees::AbstractVector{Node{T}}, dataset::Dataset{T}, options::Options;
                               device::Int=0) where {T}
    h = device_dataset(dataset, device)
    dcopy = lock(() -> DEVICE_DATASETS[dataset][device], CTX_LOCK)
    GC.@preserve dataset dcopy begin
        return eval_tree_array_on(trees, h, dataset.n, options, device)
    end
end

function eval_tree_array_on(trees::AbstractVector{Node{T}}, ds::Ptr{Cvoid}, n::Int, options::Options,
                            device::Int) where {T}
    nt = length(trees)
    p = Program(trees, options, device)
    out = Matrix{T}(undef, n, nt); ok = Vector{UInt8}(undef, nt)
    try
        GC.@preserve out ok check(ccall((:srhip_eval_tree_array, libsrhip), Int32,
                                        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{UInt8}), ds, p.h, out, ok))
    finally
        destroy(p)
    end
    return out, ok .== 1
end

# ---- eval_grad_tree_array (src/InterfaceDynamicExpressions.jl:83-107) -------------
"""
    eval_grad_tree_array(tree, X, options; variable=false) -> (output, gradient, did_succeed)

variable=false: gradient[k, i] = ∂ŷ_i/∂c_k for the constants in get_constants
order (srhip_eval_grad_tree_array). variable=true: gradient[f, i] = ∂ŷ_i/∂x_f,
computed by seeding each feature leaf x_f as (x_f + c) with c = -0.0 (x + -0.0
== x bit for bit, so values and did_succeed are unchanged) and summing the
seeds' tangents per feature; needs `+` among the binary operators, else
Unsupported.
"""
function eval_grad_tree_array(tree::Node{T}, X::AbstractMatrix{T}, options::Options;
                              variable::Bool=false, device::Int=0) where {T}
    nfeat, n = size(X)
    if !variable
        value, G, ok = _const_grads(tree, X, options, device)
        return value, permutedims(G), ok
    end
    plus = findfirst(op -> op === (+), options.operators.binops)
    plus === nothing && throw(Unsupported("variable=true needs + among the binary operators"))
    seeds = Int[]
    function seed(t::Node{T})
        if t.degree == 0
            t.constant && (push!(seeds, 0); return Node(T; val=t.val))
            push!(seeds, t.feature)
            return Node(plus, Node(T; feature=t.feature), Node(T; val=T(-0.0)))
        elseif t.degree == 1
            return Node(t.op, seed(t.l))
        else
            l = seed(t.l)
            return Node(t.op, l, seed(t.r))
        end
    end
    aug = seed(tree)
    value, G, ok = _const_grads(aug, X, options, device)
    grad = zeros(T, nfeat, n)
    for (k, f) in enumerate(seeds)
        f > 0 && (grad[f, :] .+= view(G, :, k))
    end
    return value, grad, ok
end

function _const_grads(tree::Node{T}, X::AbstractMatrix{T}, options::Options, device::Int) where {T}
    n = size(X, 2)
    ds = upload(X, zeros(T, n), nothing, device)
    p = Program([tree], options, device)
    ncon = Int(p.const_off[end])
    value = Vector{T}(undef, n); G = Matrix{T}(undef, n, ncon); ok = Ref{UInt8}(0)
    try
        GC.@preserve value G check(ccall((:srhip_eval_grad_tree_array, libsrhip), Int32,
                                         (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ref{UInt8}),
                                         ds, p.h, value, G, ok))
    finally
        destroy(p)
        destroy_dataset(ds)
    end
    return value, G, ok[] == 1
end

end # module
