"""Offline (single-process) plan generation equals the collective builder on every rank,
and saved plans round-trip through ``torch.load(weights_only=True)``."""
import pytest
import torch

from dgraph_amd.plan.pattern import (build_all_patterns_offline, build_communication_pattern,
                                     load_pattern, save_patterns)


def _graph(V=40, E=220, seed=1):
    g = torch.Generator().manual_seed(seed)
    e = torch.randint(0, V, (E, 2), generator=g)
    e = torch.cat([e, e.flip(1)])
    return torch.unique(e, dim=0), torch.randint(0, 3, (V,), generator=g)


def _compare(rank, world, tmpdir):
    E, part = _graph()
    part = part % world
    online = build_communication_pattern(E, part, rank, world)
    offline = build_all_patterns_offline(E, part, world)[rank]
    for name in ("local_edge_list", "send_local_idx", "send_offset", "recv_offset", "comm_map",
                 "put_forward_remote_offset", "put_backward_remote_offset", "halo_vertices"):
        a, b = getattr(online, name), getattr(offline, name)
        assert torch.equal(a.cpu().long(), b.cpu().long()), name
    assert online.num_halo_vertices == offline.num_halo_vertices
    if rank == 0:
        save_patterns(build_all_patterns_offline(E, part, world), tmpdir, "g")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_offline_patterns_match_collective(ranks, world, tmp_path):
    ranks(_compare, world, str(tmp_path))
    E, part = _graph()
    ref = build_all_patterns_offline(E, part % world, world)
    for r in range(world):
        cp = load_pattern(str(tmp_path), "g", r, world)
        assert torch.equal(cp.send_local_idx.long(), ref[r].send_local_idx.long())
        assert cp.send_splits() == ref[r].send_splits()
        assert cp.recv_splits() == ref[r].recv_splits()
