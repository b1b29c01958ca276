# SRHip.jl — the Julia side of the drop-in boundary (ccall into libsrhip.so).
#
# This is the binding a SymbolicRegression.jl maintainer would add; Julia is
# not available in this build image, so it is not executed here (the C ABI it
# calls is tested from Python, tests/test_abi.py and tests/test_gpu_parity.py).
# See INTEGRATION.md for where it plugs into the reference.
module SRHip

using DynamicExpressions: Node
import ..CoreModule: Options, Dataset

const libsrhip = get(ENV, "SRHIP_LIB", joinpath(@__DIR__, "..", "lib", "libsrhip.so"))

const SRHIP_OK = Int32(0)
const SRHIP_ERR_UNSUPPORTED = Int32(-2)
const NODE_CONST, NODE_FEATURE, NODE_UNARY, NODE_BINARY = UInt8(0), UInt8(1), UInt8(2), UInt8(3)
const LOSS_L2, LOSS_L1, LOSS_LP, LOSS_HUBER = Int32(0), Int32(1), Int32(2), Int32(3)

struct SrhipTrees              # include/srhip.h: srhip_trees
    ntrees::Int32
    node_off::Ptr{Int32}
    kind::Ptr{UInt8}
    arg::Ptr{UInt16}
    const_off::Ptr{Int32}
    consts::Ptr{Cvoid}
end

struct Unsupported <: Exception
    msg::String
end

last_error() = unsafe_string(ccall((:srhip_last_error, libsrhip), Cstring, ()))
function check(rc::Int32)
    rc == SRHIP_OK && return nothing
    rc == SRHIP_ERR_UNSUPPORTED && throw(Unsupported(last_error()))
    error("srhip: $(last_error())")
end

dtype_code(::Type{Float32}) = Int32(0)
dtype_code(::Type{Float64}) = Int32(1)
dtype_code(::Type) = throw(Unsupported("only Float32/Float64 run on the GPU"))

# one context per (thread, device): calls through a context are serialised
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

# operator ids, once per Options (srhip_op_lookup applies binopmap/unaopmap names)
function op_id(op, arity)
    a = Ref{Int32}(0); i = Ref{Int32}(0)
    check(ccall((:srhip_op_lookup, libsrhip), Int32, (Cstring, Ptr{Int32}, Ptr{Int32}),
                string(nameof(op)), a, i))
    a[] == arity || throw(Unsupported("operator $(op) has arity $(a[])"))
    return UInt16(i[])
end
operator_ids(options::Options) = (
    [op_id(op, 2) for op in options.operators.binops],
    [op_id(op, 1) for op in options.operators.unaops],
)

# post-order flattening; constants in get_constants order
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

# device copy of a Dataset, uploaded once (src/Dataset.jl:24-64)
const DEVICE_DATASETS = IdDict{Any,Ptr{Cvoid}}()
function device_dataset(dataset::Dataset{T}, device::Int=0) where {T}
    get!(DEVICE_DATASETS, dataset) do
        h = Ref{Ptr{Cvoid}}(C_NULL)
        X = Matrix{T}(dataset.X); y = Vector{T}(dataset.y)
        w = dataset.weighted ? Vector{T}(dataset.weights) : nothing
        GC.@preserve X y w begin
            check(ccall((:srhip_dataset_create, libsrhip), Int32,
                        (Ptr{Cvoid}, Int32, Int32, Ptr{T}, Ptr{T}, Ptr{T}, Int64, Int32, Int64, Int64,
                         Ptr{Ptr{Cvoid}}),
                        context(device), dtype_code(T), Int32(0), X, y,
                        w === nothing ? Ptr{T}(C_NULL) : w, dataset.n, dataset.nfeatures, 0, dataset.n, h))
        end
        h[]
    end
end

loss_code(::Any) = throw(Unsupported("elementwise loss not in the engine's table"))
# (the shim maps L2DistLoss/L1DistLoss/LPDistLoss/HuberLoss/... to SRHIP_LOSS_*)

"""
    eval_loss_batch(trees, dataset, options) -> Vector{T}

Batched `eval_loss` (src/LossFunctions.jl:60-67): one device launch for all
trees; T(Inf) where evaluation fails.
"""
function eval_loss_batch(trees::AbstractVector{Node{T}}, dataset::Dataset{T}, options::Options;
                         idx=nothing) where {T}
    node_off, kind, arg, const_off, consts = flatten(trees, options)
    nt = length(trees)
    sums = Vector{Float64}(undef, nt); ok = Vector{UInt8}(undef, nt); wsum = Ref{Float64}(0)
    kindcode, param = loss_code(options.elementwise_loss)
    params = Float64[param]
    rows = idx === nothing ? Int64[] : Int64.(idx .- 1)
    GC.@preserve node_off kind arg const_off consts sums ok params rows begin
        tr = Ref(SrhipTrees(nt, pointer(node_off), pointer(kind), pointer(arg), pointer(const_off),
                            Ptr{Cvoid}(pointer(consts))))
        check(ccall((:srhip_eval_loss_batch, libsrhip), Int32,
                    (Ptr{Cvoid}, Ref{SrhipTrees}, Int32, Ptr{Float64}, Ptr{Int64}, Int64, Ptr{Float64},
                     Ref{Float64}, Ptr{UInt8}),
                    device_dataset(dataset), tr, kindcode, params,
                    idx === nothing ? Ptr{Int64}(C_NULL) : pointer(rows), length(rows), sums, wsum, ok))
    end
    return [ok[i] == 1 ? T(sums[i] / wsum[]) : T(Inf) for i in 1:nt]
end

end # module
