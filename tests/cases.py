"""Hand-derived gossip cases shared by the oracle tests (CPU) and the engine tests (GPU).

Each case is a replay: explicit link keys, explicit counted generations, the expected
per-node counters derived by hand from the reference's rules (p2pnode.cc:127-199):
first arrival -> received/forwarded + send to every peer (sender and duplicates included);
later arrivals are dropped; a generation always counts and always sends, even when the id
was already seen.  L = 5 ms, t_start = 5 s.
"""
L = 5_000_000
T0 = 5_000_000_000
BIG = T0 + 50 * L  # far past the end of every flood in these cases


def case(name, n, links, events, t_cut, expect):
    return dict(name=name, n=n, links=links, events=events, t_cut=t_cut, expect=expect)


t = T0 + 123_457  # a generation phase inside the first tick

CASES = [
    # path 0-1-2, one share from node 0
    case("path", 3, [(0, 1), (1, 2)], [(t, 0, 7)], BIG,
         dict(gen=[1, 0, 0], recv=[0, 1, 1], sent=[1, 2, 1], processed=[1, 1, 1])),
    # cut between hop 1 and hop 2: node 2's arrival (t + 2L) is after PrintStatistics
    case("path_cut", 3, [(0, 1), (1, 2)], [(t, 0, 7)], t + L + L // 2,
         dict(gen=[1, 0, 0], recv=[0, 1, 0], sent=[1, 2, 0], processed=[1, 1, 0])),
    # an arrival exactly at t_cut is not counted (PrintStatistics was scheduled first)
    case("path_cut_exact", 3, [(0, 1), (1, 2)], [(t, 0, 7)], t + 2 * L,
         dict(gen=[1, 0, 0], recv=[0, 1, 0], sent=[1, 2, 0], processed=[1, 1, 0])),
    # parallel link (0,1)+(1,0): both ends see each other twice -> 2 sends each
    case("parallel", 3, [(0, 1), (1, 0), (1, 2)], [(t, 0, 9)], BIG,
         dict(gen=[1, 0, 0], recv=[0, 1, 1], sent=[2, 3, 1], processed=[1, 1, 1])),
    # same id generated at nodes 0 and 2 (collision), node 2 generates before the flood
    # from node 0 reaches it: both generations effective, node 1 receives once
    case("collide_both_effective", 3, [(0, 1), (1, 2)], [(t, 0, 5), (t + L // 2, 2, 5)], BIG,
         dict(gen=[1, 0, 1], recv=[0, 1, 0], sent=[1, 2, 1], processed=[1, 1, 1])),
    # node 2 generates the id after it already received it: gen+send count, no new process
    case("collide_after_receive", 3, [(0, 1), (1, 2)], [(t, 0, 5), (t + 3 * L, 2, 5)], BIG,
         dict(gen=[1, 0, 1], recv=[0, 1, 1], sent=[1, 2, 2], processed=[1, 1, 1])),
    # generation at the very ns the flood arrives: the generation event was scheduled
    # earlier, so it runs first and the arrival is a duplicate
    case("collide_tie", 3, [(0, 1), (1, 2)], [(t, 0, 5), (t + 2 * L, 2, 5)], BIG,
         dict(gen=[1, 0, 1], recv=[0, 1, 0], sent=[1, 2, 1], processed=[1, 1, 1])),
    # same-tick race at node 2: its own generation (phase later) loses to the arrival
    case("collide_same_tick_arrival_first", 3, [(0, 1), (1, 2)],
         [(t, 0, 5), (t + 2 * L + 1000, 2, 5)], BIG,
         dict(gen=[1, 0, 1], recv=[0, 1, 1], sent=[1, 2, 2], processed=[1, 1, 1])),
    # same-tick race at node 2 where its generation phase is earlier than the arrival's
    case("collide_same_tick_gen_first", 3, [(0, 1), (1, 2)],
         [(t, 0, 5), (t + 2 * L - 1000, 2, 5)], BIG,
         dict(gen=[1, 0, 1], recv=[0, 1, 0], sent=[1, 2, 1], processed=[1, 1, 1])),
    # same id in two components: independent floods, no interaction
    case("collide_two_components", 4, [(0, 1), (2, 3)], [(t, 0, 5), (t + 7 * L, 2, 5)], BIG,
         dict(gen=[1, 0, 1, 0], recv=[0, 1, 0, 1], sent=[1, 1, 1, 1], processed=[1, 1, 1, 1])),
    # two colliding floods meeting in the middle of a path 0-1-2-3-4 (same phase offset):
    # node 2 is reached by both at t + 2L; node 1 by 0's, node 3 by 4's
    case("collide_meet", 5, [(0, 1), (1, 2), (2, 3), (3, 4)], [(t, 0, 3), (t + 100, 4, 3)], BIG,
         dict(gen=[1, 0, 0, 0, 1], recv=[0, 1, 1, 1, 0], sent=[1, 2, 2, 2, 1],
              processed=[1, 1, 1, 1, 1])),
]
