"""The native node search (dpow_node_mine) and the coverage exit of a bounded search, against
the oracle, on the GPU.

A rank of a G-GPU node searches its partition (worker_byte = rank, worker_bits = log2 G;
coordinator.go:127,326) and stops at another rank's posted hit: since round 5 it returns as
soon as the posted index lies within what its consumed launches cover, without waiting for the
launches still in flight.  The invariant that must hold whenever the post lands: a rank never
skips a hit of its own below the posted index.  Each case runs one rank in this process over a
local board (votes = NULL: the rank's values alone), with a post at a random moment from the
emulation's poster thread (dpow_diag_node_post_at), and checks the result against the oracle's
first hit of the rank's partition (worker.go:301-400 restated, oracle/dpow_oracle.c):

- post = the node's true first hit g (the workerBits = 0 answer): the rank answers g (posted,
  or its own if it is the owner) or its own first hit h_r if that was found before the post;
- post = h_r + d, a bogus "hit" above the rank's own first hit: the rank must answer h_r.
"""
import random
import time

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle():
    from _oracle import Oracle
    return Oracle()


def _cases(seed=20261018, count=10):
    rng = random.Random(seed)
    return [([rng.randrange(256) for _ in range(4)], rng.choice((4, 5)), rng.choice((2, 4))) for _ in range(count)]


def _posts_vs_oracle(oracle, cases, k_end, delays_us=(0, 60)):
    import distpow
    from distpow.node import NodeBoard, node_mine

    L = distpow.lib()
    board = NodeBoard.local()
    checked = 0
    try:
        with distpow.Miner(0) as m:
            for nonce, ntz, world in cases:
                b = world.bit_length() - 1
                g = oracle.mine_window(nonce, ntz, 0, 0, 0, k_end)[1]
                for rank in range(world):
                    hit = oracle.mine_window(nonce, ntz, rank, b, 0, k_end)
                    assert hit is not None
                    h = hit[1]
                    for post, delay_us in ((g, random.randrange(*delays_us)),
                                           (h + random.randrange(1, 1 << 20), random.randrange(*delays_us))):
                        slot = board.begin()
                        L.dpow_diag_node_post_at(slot, post, time.perf_counter_ns() + delay_us * 1000)
                        r = node_mine(None, nonce, ntz, rank, world, board=board, miner=m)
                        time.sleep(2e-4)  # a post timed after the search's end lands before the slot's reuse
                        assert r.status == distpow.FOUND, (nonce, ntz, world, rank, post, r)
                        if post == g:
                            assert r.global_idx in (g, h), (nonce, ntz, world, rank, g, h, r.global_idx)
                        else:  # a bogus post above this rank's own first hit: never taken for coverage
                            assert r.global_idx == h, (nonce, ntz, world, rank, h, post, r.global_idx)
                        assert r.secret == distpow.secret_from_index(r.global_idx)
                        assert distpow.verify(nonce, r.secret, ntz)
                        checked += 1
    finally:
        board.close()
    return checked


def test_native_rank_search_with_posts_vs_oracle(oracle):
    # k_end: the oracle stops at the first hit (16^N / R k expected)
    assert _posts_vs_oracle(oracle, _cases(), 1 << 20, (0, 60)) >= 40


def test_native_rank_search_posts_across_launches_vs_oracle(oracle):
    """the coverage exit (a post at or below what the consumed launches cover ends a
    search) where a rank's window runs several launches, queued kDepth ahead, when the post
    lands: 5- and 7-byte nonces (no chunk-length-spanning launch: the window splits at k = 256
    and 65536, and each rank's first hit lies past k = 256), N = 5, world 2 and 4, the node's true
    first hit and bogus posts above a rank's own first hit at random moments of its search."""
    rng = random.Random(20261019)
    cases = [([rng.randrange(256) for _ in range(nlen)], 5, world)
             for world in (2, 4) for nlen in (5, 7) for _ in range(2)]
    assert _posts_vs_oracle(oracle, cases, 1 << 20, (0, 80)) >= 48


def test_search_returns_at_covered_bound_vs_oracle(oracle):
    """dpow_search on an attached slot, a bound posted before the start and inside the window:
    EXHAUSTED exactly when the partition has no hit below the bound, else that first hit."""
    import distpow
    from distpow.node import NodeBoard

    board = NodeBoard.local()
    rng = random.Random(7)
    try:
        with distpow.Miner(0) as m:
            for _ in range(12):
                nonce = [rng.randrange(256) for _ in range(4)]
                ntz, world = 4, rng.choice((2, 4))
                b = world.bit_length() - 1
                rank = rng.randrange(world)
                h = oracle.mine_window(nonce, ntz, rank, b, 0, 1 << 20)[1]
                bound = h + rng.choice((-1, 1)) * rng.randrange(1, 1 << 16)
                bound = max(1, bound)
                slot = board.begin()
                distpow.lib().dpow_node_slot_reset(slot)
                distpow.lib().dpow_node_post(slot, bound)
                m.attach_node(slot)
                try:
                    r = m.search(nonce, ntz, rank, b, 0, 1 << 20)
                finally:
                    m.attach_node(None)
                    board.end()
                if h < bound:
                    assert r.status == distpow.FOUND and r.global_idx == h, (nonce, rank, world, h, bound, r)
                else:
                    assert r.status == distpow.EXHAUSTED, (nonce, rank, world, h, bound, r)
    finally:
        board.close()
