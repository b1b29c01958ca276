# BatchedCallers.jl — the hot path's callers, batched (SURVEY.md §8 a10 / f1).
#
# The reference scores one candidate at a time: next_generation
# (src/Mutate.jl:26-255) calls score_func per mutated tree inside
# reg_evol_cycle (src/RegularizedEvolution.jl:13-155), Population(...)
# (src/Population.jl:31-46) and finalize_scores (:134-148) score member by
# member. This module keeps those algorithms and moves the scoring out of the
# per-candidate loop, so that one SRHip.eval_loss_batch launch scores every
# candidate of a step:
#
#   * `population_batched`      — Population(dataset; npop, nlength, options, nfeatures)
#   * `finalize_scores_batched` — finalize_scores(dataset, pop, options)
#   * `reg_evol_cycle_lockstep` — reg_evol_cycle with the reference's DEFAULT
#     semantics (fast_cycle = false: best_of_sample, next_generation or
#     crossover_generation, replace-oldest, step by step per island), every
#     island's candidates of a step — both crossover children included — in
#     one launch; `s_r_cycle_lockstep` runs a whole s_r_cycle that way.
#   * `reg_evol_cycle_batched`  — reg_evol_cycle with fast_cycle semantics
#     (one baby per tournament_selection_n-member subsample, replace-oldest),
#     for several islands in lockstep: every island's babies in one launch,
#     and every `:optimize` mutation of the cycle in one batched optimiser call.
#   * `optimize_constants_batched` — optimize_constants (src/ConstantOptimization.jl:22-65)
#     for many members: SRHip.optimize_constants_batch! (srhip_optimize_constants_batch,
#     all starts of all members in lockstep, one launch per phase).
#   * `optimize_and_simplify_population_batched` — optimize_and_simplify_population
#     (src/SingleIteration.jl:63-123): the members drawn for optimisation go
#     through one batched optimiser call instead of one Optim run each.
#
# next_generation is split into `propose` (mutation choice, attempts,
# check_constraints — everything before score_func, calling the reference's
# own mutation functions) and `accept` (the NaN rejection and the
# annealing / adaptive-parsimony acceptance rule after it). A candidate whose
# mutation needs no score (simplify, optimize, do_nothing, a failed
# constraint check) is decided in `propose`, as in the reference.
#
# UNTESTED AS JULIA (no Julia in the build image). The Python mirrors of the
# same lockstep loops (symbolicregression.jl_amd/srhip/evolution.py for the
# default path, srhip/search.py for fast_cycle) run in the test suite; tests/test_julia_binding.py checks this file's references to
# the reference's functions and to SRHip statically.
module BatchedCallers

import DynamicExpressions: Node, copy_node, count_constants, count_depth, simplify_tree, combine_operators
import ..CoreModule: Options, Dataset, RecordType, sample_mutation
import ..ComplexityModule: compute_complexity
import ..LossFunctionsModule: score_func, score_func_batch, loss_to_score
import ..CheckConstraintsModule: check_constraints
import ..AdaptiveParsimonyModule: RunningSearchStatistics
import ..PopMemberModule: PopMember, copy_pop_member
import ..PopulationModule: Population, best_of_sample
import ..HallOfFameModule: HallOfFame
import ..MutationFunctionsModule:
    gen_random_tree, gen_random_tree_fixed_size, mutate_constant, mutate_operator, append_random_op,
    prepend_random_op, insert_random_op, delete_random_op, crossover_trees
import ..ConstantOptimizationModule: optimize_constants
import ..UtilsModule: get_birth_order
import ..PopMemberModule: generate_reference
import ..RecorderModule: @recorder
import ..SingleIterationModule: s_r_cycle
import DynamicExpressions: string_tree
import ..SRHip

"""
    score_batch(dataset, trees, options) -> (scores, losses)

score_func (src/LossFunctions.jl:86-92) for every tree: one SRHip launch when
the engine covers the options, else the reference, tree by tree.
"""
function score_batch(dataset::Dataset{T}, trees::AbstractVector{Node{T}}, options::Options) where {T}
    if !isempty(trees) && SRHip.enabled(options)
        try
            losses = SRHip.eval_loss_batch(trees, dataset, options)
            scores = [loss_to_score(l, dataset.baseline_loss, t, options) for (l, t) in zip(losses, trees)]
            return scores, losses
        catch e
            e isa SRHip.Unsupported || rethrow()
        end
    end
    pairs = [score_func(dataset, t, options) for t in trees]
    return T[p[1] for p in pairs], T[p[2] for p in pairs]
end

"""
    score_batch_minibatch(dataset, trees, options) -> (scores, losses)

score_func_batch (src/LossFunctions.jl:95-115) for every tree: each tree on
its OWN sample of batch_size rows drawn with replacement, as the reference
draws one per call (:98), all trees in one launch
(SRHip.eval_loss_batch_rowsets); a failed evaluation scores (0, Inf) as in
the reference.
"""
function score_batch_minibatch(dataset::Dataset{T}, trees::AbstractVector{Node{T}}, options::Options) where {T}
    if !isempty(trees) && SRHip.enabled(options)
        try
            idx = rand(1:(dataset.n), options.batch_size, length(trees))  # column t: tree t's sample
            losses = SRHip.eval_loss_batch_rowsets(trees, dataset, options, idx)
            scores = [isfinite(l) ? loss_to_score(l, dataset.baseline_loss, t, options) : zero(T)
                      for (l, t) in zip(losses, trees)]
            return scores, losses
        catch e
            e isa SRHip.Unsupported || rethrow()
        end
    end
    pairs = [score_func_batch(dataset, t, options) for t in trees]
    return T[p[1] for p in pairs], T[p[2] for p in pairs]
end

# ---- Population / finalize_scores ---------------------------------------------------

"""Population(dataset; npop, nlength, options, nfeatures) with one launch."""
function population_batched(dataset::Dataset{T}; npop::Int, nlength::Int=3, options::Options,
                            nfeatures::Int) where {T}
    trees = [gen_random_tree(nlength, options, nfeatures, T) for _ in 1:npop]
    scores, losses = score_batch(dataset, trees, options)
    members = [PopMember(trees[i], scores[i], losses[i]; parent=-1, deterministic=options.deterministic)
               for i in 1:npop]
    return Population{T}(members, npop)
end

"""finalize_scores (src/Population.jl:134-148): with batching, every member is
re-scored on the full dataset — one launch for the population."""
function finalize_scores_batched(dataset::Dataset{T}, pop::Population, options::Options) where {T}
    options.batching || return (pop, 0.0)
    scores, losses = score_batch(dataset, [m.tree for m in pop.members], options)
    for (m, s, l) in zip(pop.members, scores, losses)
        m.score = s
        m.loss = l
    end
    return (pop, pop.n * (options.batch_size / dataset.n))
end

# ---- constant optimisation ---------------------------------------------------------------

"""
    optimize_constants_batched(dataset, members, options) -> num_evals::Vector{Float64}

optimize_constants (src/ConstantOptimization.jl:22-65) for every member at once,
updated in place: a converged member gets the optimised constants, its
score_func re-score (:58) and a new birth (:60); the others keep x0 (:62).
One SRHip call when the engine covers the options, else the reference member
by member.
"""
function optimize_constants_batched(dataset::Dataset{T}, members::AbstractVector{<:PopMember{T}},
                                    options::Options) where {T}
    isempty(members) && return Float64[]
    if SRHip.enabled(options)
        try
            trees = Node{T}[m.tree for m in members]
            losses, converged, num_evals = SRHip.optimize_constants_batch!(trees, dataset, options)
            for (m, l, c) in zip(members, losses, converged)
                c || continue
                m.score = loss_to_score(l, dataset.baseline_loss, m.tree, options)
                m.loss = l
                m.birth = get_birth_order(; deterministic=options.deterministic)
            end
            return num_evals
        catch e
            e isa SRHip.Unsupported || rethrow()
        end
    end
    evals = zeros(Float64, length(members))
    for (j, m) in enumerate(members)
        _, evals[j] = optimize_constants(dataset, m, options)
    end
    return evals
end

"""
    optimize_and_simplify_population_batched(dataset, pop, options, curmaxsize, record) -> (pop, num_evals)

optimize_and_simplify_population (src/SingleIteration.jl:63-123) with the
members drawn for optimisation (rand(pop.n) .< optimizer_probability)
optimised in one batched call and finalize_scores as one launch; the
simplification, the new references and the record are the reference's.
"""
function optimize_and_simplify_population_batched(dataset::Dataset{T}, pop::Population, options::Options,
                                                  curmaxsize::Int, record::RecordType) where {T}
    do_optimization = rand(pop.n) .< options.optimizer_probability
    for j in 1:(pop.n)
        pop.members[j].tree = simplify_tree(pop.members[j].tree, options.operators)
        pop.members[j].tree = combine_operators(pop.members[j].tree, options.operators)
    end
    chosen = options.should_optimize_constants ? findall(do_optimization) : Int[]
    num_evals = sum(optimize_constants_batched(dataset, pop.members[chosen], options); init=0.0)
    pop, tmp_num_evals = finalize_scores_batched(dataset, pop, options)
    num_evals += tmp_num_evals
    for j in 1:(pop.n)
        old_ref = pop.members[j].ref
        new_ref = generate_reference()
        pop.members[j].parent = old_ref
        pop.members[j].ref = new_ref
        @recorder begin
            @assert haskey(record, "mutations")
            member = pop.members[j]
            if !haskey(record["mutations"], "$(member.ref)")
                record["mutations"]["$(member.ref)"] = RecordType(
                    "events" => Vector{RecordType}(), "tree" => string_tree(member.tree, options.operators),
                    "score" => member.score, "loss" => member.loss, "parent" => member.parent)
            end
            kind = (do_optimization[j] && options.should_optimize_constants) ? "simplification_and_optimization" :
                   "simplification"
            push!(record["mutations"]["$(old_ref)"]["events"],
                  RecordType("type" => "tuning", "time" => time(), "child" => new_ref,
                             "mutation" => RecordType("type" => kind)))
            push!(record["mutations"]["$(old_ref)"]["events"], RecordType("type" => "death", "time" => time()))
        end
    end
    return (pop, num_evals)
end

# ---- next_generation, split around its score_func call ---------------------------------

# A proposal: either decided (`member` set: no score needed) or a tree to score.
struct Proposal{T}
    parent::PopMember{T}
    tree::Union{Node{T},Nothing}
    member::Union{PopMember{T},Nothing}
    accepted::Bool
    num_evals::Float64
    # beforeScore / beforeLoss (src/Mutate.jl:41-47): the parent's own, or with
    # options.batching its re-score on a fresh minibatch
    before_score::T
    before_loss::T
    # an `:optimize` mutation (src/Mutate.jl:147-152): `member` holds the copy to
    # optimise; reg_evol_cycle_batched optimises all of them in one batched call
    optimize::Bool
end
Proposal{T}(parent, tree, member, accepted, num_evals, bs, bl) where {T} =
    Proposal{T}(parent, tree, member, accepted, num_evals, bs, bl, false)

# the tree-producing mutations of next_generation (src/Mutate.jl:79-115,132-139),
# through the reference's own mutation functions
function mutate_tree(choice::Symbol, tree::Node{T}, temperature, curmaxsize::Int, options::Options,
                     nfeatures::Int) where {T}
    choice == :mutate_constant && return mutate_constant(tree, temperature, options)
    choice == :mutate_operator && return mutate_operator(tree, options)
    choice == :add_node && return rand() < 0.5 ? append_random_op(tree, options, nfeatures) :
                                                 prepend_random_op(tree, options, nfeatures)
    choice == :insert_node && return insert_random_op(tree, options, nfeatures)
    choice == :delete_node && return delete_random_op(tree, options, nfeatures)
    choice == :randomize && return gen_random_tree_fixed_size(rand(1:curmaxsize), options, nfeatures, T)
    error("Unknown mutation choice: $choice")
end

"""Everything of next_generation before score_func (src/Mutate.jl:26-193);
`before` = (beforeScore, beforeLoss), already re-scored on a minibatch by the
caller when options.batching (:41-47)."""
function propose(dataset::Dataset{T}, member::PopMember{T}, before::Tuple{T,T}, temperature,
                 curmaxsize::Int, options::Options) where {T}
    prev = member.tree
    bs, bl = before
    keep(tree, accepted, evals=0.0) = Proposal{T}(member, nothing,
        PopMember(tree, bs, bl; parent=member.ref, deterministic=options.deterministic),
        accepted, evals, bs, bl)
    weights = copy(options.mutation_weights)
    weights.mutate_constant *= min(8, count_constants(prev)) / 8.0
    if compute_complexity(prev, options) >= curmaxsize || count_depth(prev) >= options.maxdepth
        weights.add_node = 0.0
        weights.insert_node = 0.0
    end
    choice = sample_mutation(weights)
    choice == :do_nothing && return keep(prev, true)
    if choice == :simplify
        return keep(combine_operators(simplify_tree(copy_node(prev), options.operators), options.operators), true)
    end
    if choice == :optimize  # optimised with the cycle's other :optimize proposals (reg_evol_cycle_batched)
        m = PopMember(copy_node(prev), bs, bl; parent=member.ref, deterministic=options.deterministic)
        return Proposal{T}(member, nothing, m, true, 0.0, bs, bl, true)
    end
    for _ in 1:10  # max_attempts
        tree = mutate_tree(choice, copy_node(prev), temperature, curmaxsize, options, dataset.nfeatures)
        check_constraints(tree, options, curmaxsize) &&
            return Proposal{T}(member, tree, nothing, false, 0.0, bs, bl)
    end
    return keep(copy_node(prev), false)  # failed constraint check: rejected
end

"""Everything of next_generation after score_func (src/Mutate.jl:207-255)."""
function accept(p::Proposal{T}, score::T, loss::T, temperature, stats::RunningSearchStatistics,
                options::Options) where {T}
    member = p.parent
    reject() = (PopMember(copy_node(member.tree), p.before_score, p.before_loss; parent=member.ref,
                          deterministic=options.deterministic), false)
    isnan(score) && return reject()
    prob = 1.0
    if options.annealing
        prob *= exp(-(score - p.before_score) / (temperature * options.alpha))
    end
    if options.use_frequency
        freq(c) = 0 < c <= options.maxsize ? stats.normalized_frequencies[c] : 1e-6
        prob *= freq(compute_complexity(member.tree, options)) / freq(compute_complexity(p.tree, options))
    end
    prob < rand() && return reject()
    return (PopMember(p.tree, score, loss; parent=member.ref, deterministic=options.deterministic), true)
end

# ---- reg_evol_cycle, fast_cycle semantics, islands in lockstep ------------------------

"""
    reg_evol_cycle_batched(dataset, pops, temperature, curmaxsize, stats, options) -> (pops, num_evals)

One fast_cycle pass (src/RegularizedEvolution.jl:33-79) over every island
of `pops` at once: shuffle each population, take the best of every
tournament_selection_n-member subsample, propose one baby each, score ALL
islands' babies in one launch, then accept and replace the oldest member
per island, in the reference's order.
"""
function reg_evol_cycle_batched(dataset::Dataset{T}, pops::AbstractVector{<:Population}, temperature,
                                curmaxsize::Int, stats::AbstractVector{RunningSearchStatistics},
                                options::Options) where {T}
    proposals = Vector{Vector{Proposal{T}}}(undef, length(pops))
    allstars = Vector{Vector{PopMember{T}}}(undef, length(pops))
    for (k, pop) in enumerate(pops)
        shuffle!(pop.members)
        ncyc = round(Int, pop.n / options.tournament_selection_n)
        allstars[k] = [begin
                           sub = (1 + (i - 1) * options.tournament_selection_n):(i * options.tournament_selection_n)
                           pop.members[sub[argmin([pop.members[j].score for j in sub])]]
                       end for i in 1:ncyc]
    end
    # with options.batching, every next_generation first re-scores its parent
    # on a minibatch (src/Mutate.jl:41-47): one launch for all islands' parents
    parents = PopMember{T}[m for as in allstars for m in as]
    num_evals = 0.0
    before = if options.batching
        ps, pl = score_batch_minibatch(dataset, Node{T}[m.tree for m in parents], options)
        num_evals += length(parents) * (options.batch_size / dataset.n)
        collect(zip(ps, pl))
    else
        [(m.score, m.loss) for m in parents]
    end
    q = 0
    for (k, as) in enumerate(allstars)
        props = Vector{Proposal{T}}(undef, length(as))
        off = q
        Threads.@threads for i in eachindex(as)
            props[i] = propose(dataset, as[i], before[off + i], temperature, curmaxsize, options)
        end
        q += length(as)
        proposals[k] = props
    end
    # every :optimize mutation of every island in one batched optimiser call
    to_opt = PopMember{T}[p.member for props in proposals for p in props if p.optimize]
    num_evals += sum(optimize_constants_batched(dataset, to_opt, options); init=0.0)
    # one launch for every island's babies
    trees = Node{T}[p.tree for props in proposals for p in props if p.member === nothing]
    scores, losses = options.batching ? score_batch_minibatch(dataset, trees, options) :
                     score_batch(dataset, trees, options)
    num_evals += length(trees) * (options.batching ? options.batch_size / dataset.n : 1.0)
    j = 0
    for (k, pop) in enumerate(pops)
        for p in proposals[k]
            num_evals += p.num_evals
            baby, accepted = if p.member === nothing
                j += 1
                accept(p, scores[j], losses[j], temperature, stats[k], options)
            else
                (p.member, p.accepted)
            end
            oldest = argmin([m.birth for m in pop.members])
            (accepted || !options.skip_mutation_failures) && (pop.members[oldest] = baby)
        end
    end
    return pops, num_evals
end

shuffle!(v) = (for i in length(v):-1:2; j = rand(1:i); v[i], v[j] = v[j], v[i]; end; v)

# ---- reg_evol_cycle, DEFAULT semantics (fast_cycle = false), islands in lockstep ----------

# One island's step in flight: a mutation (Proposal) or a crossover pair.
struct Step{T}
    crossover::Bool
    prop::Union{Proposal{T},Nothing}        # mutation: next_generation's proposal
    parents::Tuple{Vararg{PopMember{T}}}     # crossover: (allstar1, allstar2)
    children::Union{Tuple{Node{T},Node{T}},Nothing}  # crossover children; nothing = failed constraints
end

"""
    crossover_children(m1, m2, curmaxsize, options) -> (child1, child2) or nothing

crossover_generation (src/Mutate.jl:285-313) up to its score_func calls:
crossover_trees until both children pass check_constraints, at most 11 tries.
"""
function crossover_children(m1::PopMember{T}, m2::PopMember{T}, curmaxsize::Int, options::Options) where {T}
    c1, c2 = crossover_trees(m1.tree, m2.tree)
    num_tries = 1
    while !(check_constraints(c1, options, curmaxsize) && check_constraints(c2, options, curmaxsize))
        num_tries > 10 && return nothing
        c1, c2 = crossover_trees(m1.tree, m2.tree)
        num_tries += 1
    end
    return (c1, c2)
end

"""
    reg_evol_cycle_lockstep(dataset, pops, temperature, curmaxsize, stats, options) -> (pops, num_evals)

reg_evol_cycle with the reference's DEFAULT semantics (src/RegularizedEvolution.jl:81-155:
`fast_cycle = false`, crossover with probability `crossover_probability`,
`best_of_sample` tournaments with `tournament_selection_p`) for every island
of `pops` in lockstep. Each of the round(npop / tournament_selection_n) steps
is taken by every island together: its own `rand() > crossover_probability`
draw, `best_of_sample` (once, or twice for crossover), the mutation proposal
or the crossover children; then ALL islands' candidates — every mutated tree
and both children of every crossover — are scored in ONE launch, and each
island accepts and replaces its oldest member(s) in the reference's order.
Within an island the steps stay sequential (step i+1's tournament sees step
i's replacement), so each island runs the reference's algorithm unchanged;
`stats[k]` is island k's RunningSearchStatistics (the copy its worker holds).
The Python mirror (srhip/evolution.py) is tested to give, over the oracle,
exactly the serial per-island result.
"""
function reg_evol_cycle_lockstep(dataset::Dataset{T}, pops::AbstractVector{<:Population}, temperature,
                                 curmaxsize::Int, stats::AbstractVector{RunningSearchStatistics},
                                 options::Options) where {T}
    num_evals = 0.0
    nsteps = round(Int, pops[1].n / options.tournament_selection_n)
    for _ in 1:nsteps
        steps = Vector{Step{T}}(undef, length(pops))
        # tournaments first: each island's crossover draw and best_of_sample
        allstars = Vector{Union{PopMember{T},Nothing}}(nothing, length(pops))
        for (k, pop) in enumerate(pops)
            if rand() > options.crossover_probability
                allstars[k] = best_of_sample(pop, stats[k], options)
            else
                a1 = best_of_sample(pop, stats[k], options)
                a2 = best_of_sample(pop, stats[k], options)
                steps[k] = Step{T}(true, nothing, (a1, a2), crossover_children(a1, a2, curmaxsize, options))
            end
        end
        # with options.batching every next_generation re-scores its parent on a
        # fresh minibatch (src/Mutate.jl:41-47): all islands' parents in ONE launch,
        # each on its own sample
        mut = findall(a -> a !== nothing, allstars)
        before = if options.batching && !isempty(mut)
            ps, pl = score_batch_minibatch(dataset, Node{T}[allstars[k].tree for k in mut], options)
            num_evals += length(mut) * (options.batch_size / dataset.n)
            Dict(k => (ps[i], pl[i]) for (i, k) in enumerate(mut))
        else
            Dict(k => (allstars[k].score, allstars[k].loss) for k in mut)
        end
        for k in mut
            allstar = allstars[k]
            steps[k] = Step{T}(false, propose(dataset, allstar, before[k], temperature, curmaxsize, options),
                               (allstar,), nothing)
        end
        # every :optimize proposal of this step, all islands, in one optimiser call
        to_opt = PopMember{T}[s.prop.member for s in steps if !s.crossover && s.prop.optimize]
        num_evals += sum(optimize_constants_batched(dataset, to_opt, options); init=0.0)
        # ONE launch: mutated trees and both crossover children of every island
        trees = Node{T}[]
        for s in steps
            if s.crossover
                s.children === nothing || append!(trees, s.children)
            elseif s.prop.member === nothing
                push!(trees, s.prop.tree)
            end
        end
        scores, losses = options.batching ? score_batch_minibatch(dataset, trees, options) :
                         score_batch(dataset, trees, options)
        j = 0
        for (k, pop) in enumerate(pops)
            s = steps[k]
            if !s.crossover
                p = s.prop
                num_evals += p.num_evals
                baby, accepted = if p.member === nothing
                    j += 1
                    num_evals += options.batching ? options.batch_size / dataset.n : 1.0
                    accept(p, scores[j], losses[j], temperature, stats[k], options)
                else
                    (p.member, p.accepted)
                end
                (!accepted && options.skip_mutation_failures) && continue
                pop.members[argmin([m.birth for m in pop.members])] = baby
            else
                a1, a2 = s.parents
                if s.children === nothing
                    options.skip_mutation_failures && continue
                    b1, b2 = a1, a2  # a failed crossover returns member1, member2 (src/Mutate.jl:309)
                else
                    b1 = PopMember(s.children[1], scores[j + 1], losses[j + 1]; parent=a1.ref,
                                   deterministic=options.deterministic)
                    b2 = PopMember(s.children[2], scores[j + 2], losses[j + 2]; parent=a2.ref,
                                   deterministic=options.deterministic)
                    j += 2
                    # src/Mutate.jl:314-322: 2·batch_size/n with batching, batch_size/n without
                    num_evals += options.batching ? 2 * (options.batch_size / dataset.n) :
                                 options.batch_size / dataset.n
                end
                pop.members[argmin([m.birth for m in pop.members])] = b1
                pop.members[argmin([m.birth for m in pop.members])] = b2
            end
        end
    end
    return pops, num_evals
end

"""
    s_r_cycle_lockstep(dataset, pops, ncycles, curmaxsize, stats, options) -> (pops, best_seen, num_evals)

s_r_cycle (src/SingleIteration.jl:17-61) for every island at once: the
temperature schedule, reg_evol_cycle_lockstep (or reg_evol_cycle_batched when
options.fast_cycle), and each island's best-seen hall of fame. The head node
calls it once per round with every island it would have spawned, instead of
one @sr_spawner job per island (INTEGRATION.md §4).

With options.recorder the lockstep loops would write no genealogy (the
mutation / death events of src/RegularizedEvolution.jl:103-132), so every
island runs the reference's own s_r_cycle instead, recording into records[k].
"""
function s_r_cycle_lockstep(dataset::Dataset{T}, pops::AbstractVector{<:Population}, ncycles::Int,
                            curmaxsize::Int, stats::AbstractVector{RunningSearchStatistics},
                            options::Options; records=nothing) where {T}
    if options.recorder
        best_seen = Vector{HallOfFame{T}}(undef, length(pops))
        num_evals = 0.0
        for k in eachindex(pops)
            rec = records === nothing ? RecordType() : records[k]
            pops[k], best_seen[k], ev = s_r_cycle(dataset, pops[k], ncycles, curmaxsize, stats[k];
                                                  options=options, record=rec)
            num_evals += ev
        end
        return pops, best_seen, num_evals
    end
    max_temp = T(1.0)
    min_temp = options.annealing ? T(0.0) : max_temp
    best_seen = [HallOfFame(options, T) for _ in pops]
    num_evals = 0.0
    for temperature in LinRange(max_temp, min_temp, ncycles)
        _, ev = options.fast_cycle ?
                reg_evol_cycle_batched(dataset, pops, temperature, curmaxsize, stats, options) :
                reg_evol_cycle_lockstep(dataset, pops, temperature, curmaxsize, stats, options)
        num_evals += ev
        for (k, pop) in enumerate(pops), member in pop.members
            size = compute_complexity(member.tree, options)
            if 0 < size <= options.maxsize &&
               (!best_seen[k].exists[size] || member.score < best_seen[k].members[size].score)
                best_seen[k].exists[size] = true
                best_seen[k].members[size] = copy_pop_member(member)
            end
        end
    end
    return pops, best_seen, num_evals
end

end # module
