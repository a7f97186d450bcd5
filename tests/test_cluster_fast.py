"""cluster.sharded_spread_compiled (config (e) straight to SoA columns) against the object path:
the same cluster built as v1.Node dicts and compiled by Compiler.register + compile_snapshot must
give identical dictionaries, columns, snapshot fields and pod queries, whole and sharded."""
import numpy as np
import pytest

from kgpu import cluster, native
from kgpu.compile import Compiler, Pools

SNAP_FIELDS = ("n_nodes", "node_base", "n_total_nodes", "n_scalar", "n_label_keys", "taint_words", "port_slots",
               "n_zones", "n_pods", "n_pod_label_keys", "n_terms")


def _slow(n, n_pods, shard):
    nodes, ex, pods, prof = cluster.sharded_spread(n_nodes=n, n_pods=n_pods)
    comp = Compiler(prof)
    comp.register(nodes, ex, pods[:16])
    return comp, comp.compile_snapshot(nodes, ex, shard=shard), pods


def _queries(comp, pods):
    pools = Pools()
    qs = [comp.compile_pod(p, pools) for p in pods]
    _, pnp = pools.finalize()
    return np.array(qs), pnp


@pytest.mark.parametrize("n,world,rank", [(1, 1, 0), (7, 1, 0), (130, 1, 0), (3000, 1, 0), (3000, 4, 2),
                                          (3001, 3, 0), (3001, 3, 2)])
def test_fast_generator_matches_object_compile(n, world, rank):
    shard = None if world == 1 else native.shard_range(n, world, rank)
    c1, (s1, a1, o1), p1 = _slow(n, 40, shard)
    c2, (s2, a2, o2), p2, _ = cluster.sharded_spread_compiled(n_nodes=n, n_pods=40, shard=shard)
    assert p1 == p2
    assert o1 == o2
    assert c1.nkeys.keys.items == c2.nkeys.keys.items
    assert [d.items for d in c1.nkeys.vals] == [d.items for d in c2.nkeys.vals]
    for attr in ("taints", "zones", "ns", "scalars"):
        assert getattr(c1, attr).items == getattr(c2, attr).items, attr
    assert c1.pkeys.keys.items == c2.pkeys.keys.items
    assert [d.items for d in c1.pkeys.vals] == [d.items for d in c2.pkeys.vals]
    for f in SNAP_FIELDS:
        assert getattr(s1, f) == getattr(s2, f), f
    keys = sorted(k for k in a1 if not k.startswith("_") and isinstance(a1[k], np.ndarray))
    assert keys == sorted(k for k in a2 if not k.startswith("_") and isinstance(a2[k], np.ndarray))
    for k in keys:
        assert a1[k].dtype == a2[k].dtype and a1[k].shape == a2[k].shape, k
        assert np.array_equal(a1[k], a2[k]), k
    q1, pn1 = _queries(c1, p1)
    q2, pn2 = _queries(c2, p2)
    assert q1.tobytes() == q2.tobytes()
    for k in pn1:
        assert pn1[k].tobytes() == pn2[k].tobytes(), k


def test_fast_generator_million_nodes_is_quick():
    """The 1M-node cluster of config (e) (8 shards of 125k): one rank's shard compiles in seconds."""
    import time
    t = time.time()
    comp, (snap, arrays, order), pods, _ = cluster.sharded_spread_compiled(
        n_nodes=1_000_000, n_pods=100, shard=native.shard_range(1_000_000, 8, 3))
    assert time.time() - t < 60
    assert (snap.node_base, snap.n_nodes, snap.n_total_nodes) == (375000, 125000, 1_000_000)
    assert arrays["label_val"].shape == (2, 125000)
    assert int(arrays["label_val"][1][0]) == 375000
    assert len(order) == 1_000_000
