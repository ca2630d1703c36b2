"""fixActions beyond the golden fixtures (CPU, oracle only).

* The eviction order: the reference appends evicted agents in the iteration
  order of a CPython set intersection of (agent, action) tuples
  (mapf_gym.py:590-596).  The oracle's restatement (oc_evict_order, shared by
  the kernels' mapf_pyset.h) is checked here against this interpreter's own
  sets on random operands, built exactly as the reference builds them
  (numpy int64 tuples of agentActionPairs rows and of restrictedAction lists).
* The states the reference does not survive -- an empty viable set
  (random.choice([]) raises, :588) and a deadlock (its while loop never ends,
  :563) -- resolve to agents on distinct free cells (no swap), and are counted.
"""
import numpy as np

from oracle import oracle as O


def test_tuple_hash_matches_cpython():
    for a in range(-1, 70):
        for b in range(-1, 6):
            assert O.py_hash_pair(a, b) == hash((np.int64(a), np.int64(b))) % (1 << 64), (a, b)


def test_evict_order_matches_cpython_sets():
    rng = np.random.default_rng(0)
    multi = reordered = 0
    for _ in range(20000):
        N = int(rng.integers(2, 65))
        pairs = np.where(rng.random(N) < rng.random(), rng.integers(0, 5, N), -1)
        pairs[rng.integers(N)] = -1                     # the agent being placed is unassigned
        agent_action_pairs = np.array([[j, pairs[j]] if pairs[j] >= 0 else [-1, -1] for j in range(N)])
        js = rng.choice(N, size=int(rng.integers(1, 6)))
        restricted = sorted(set((int(j), int(pairs[j]) if (pairs[j] >= 0 and rng.random() < 0.7)
                                 else int(rng.integers(0, 5))) for j in js))
        ref = [int(x[0]) for x in set(tuple(x) for x in agent_action_pairs)
               & set(tuple(x) for x in np.array(restricted))]
        assert O.evict_order(pairs, restricted) == ref, (pairs.tolist(), restricted)
        multi += len(ref) > 1
        reordered += ref != sorted(ref)
    assert multi > 1000 and reordered > 500        # the cases where set order differs from index order


def test_deadlocks_resolve_to_distinct_cells():
    """One shared random 12x12 map (p = 0.3, largest component) with 8 agents: deadlocks
    and empty viable sets occur within a few hundred steps; agents always end on
    distinct free cells and never swap."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "primal-ppo_amd"))
    from mapf_amd.maps import keep_largest_component, random_map
    H = W = 12
    N = 8
    world = keep_largest_component(random_map(np.random.default_rng(6), H, W, 0.3))
    cfg = O.make_config(H, W, N, 11, 6, human_mode=1, goal_mode=1, fix_choice=1, keep_bfs=0, seed=77)
    free = world == 0
    counts = np.zeros(2, int)
    for b in range(48):
        e = O.OracleEnv(cfg, env_id=b)
        e.reset_random(world)
        prev, _ = e.agents()
        for _ in range(200):
            e.step(e.random_actions())
            p, _ = e.agents()
            assert free[p[:, 0], p[:, 1]].all()
            cells = p[:, 0] * W + p[:, 1]
            assert len(np.unique(cells)) == N
            pc = prev[:, 0] * W + prev[:, 1]
            for i in range(N):     # no swap: i moved onto j's old cell while j moved onto i's
                j = np.nonzero(pc == cells[i])[0]
                assert not (len(j) and j[0] != i and cells[j[0]] == pc[i])
            prev = p
        counts += e.fix_counts()
    assert counts[1] > 0 and counts[0] > 0, counts
