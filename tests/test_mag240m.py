"""MAG240M raw-layout loader (no ogb): a miniature dataset directory in the exact on-disk
layout of ogb.lsc.MAG240MDataset (meta.pt, split_dict.pt with numpy arrays, processed/*
.npy). Parity with ogb itself is unpinned (ogb is not installed); the derived author /
institution features are checked against a numpy mean, and the per-rank plan files
(MAG240M_dataset_rank_{r}_of_{W}_comm_plans.pt) against a rebuild."""
import os

import numpy as np
import pytest
import torch

NP, NA, NI, F = 50, 70, 6, 8


def make_fake_mag(root, seed=0):
    d = os.path.join(root, "mag240m_kddcup2021")
    rng = np.random.default_rng(seed)
    for sub in ("paper", "paper___cites___paper", "author___writes___paper",
                "author___affiliated_with___institution"):
        os.makedirs(os.path.join(d, "processed", sub), exist_ok=True)
    torch.save({"paper": NP, "author": NA, "institution": NI}, os.path.join(d, "meta.pt"))
    perm = rng.permutation(NP)
    torch.save({"train": perm[:30], "valid": perm[30:40], "test-dev": perm[40:45],
                "test-challenge": perm[45:]}, os.path.join(d, "split_dict.pt"))
    np.save(os.path.join(d, "processed/paper/node_feat.npy"),
            rng.standard_normal((NP, F)).astype(np.float16))
    lab = rng.integers(0, 153, NP).astype(np.float32)
    lab[perm[45:]] = np.nan
    np.save(os.path.join(d, "processed/paper/node_label.npy"), lab)
    cites = np.unique(rng.integers(0, NP, (2, 200)), axis=1)
    np.save(os.path.join(d, "processed/paper___cites___paper/edge_index.npy"), cites)
    writes = np.unique(np.stack([rng.integers(0, NA, 160), rng.integers(0, NP, 160)]), axis=1)
    np.save(os.path.join(d, "processed/author___writes___paper/edge_index.npy"), writes)
    aff = np.unique(np.stack([rng.integers(0, NA, 40), rng.integers(0, NI, 40)]), axis=1)
    np.save(os.path.join(d, "processed/author___affiliated_with___institution/edge_index.npy"),
            aff)
    return d


def _np_mean(src, edges, n_dst):
    out = np.zeros((n_dst, src.shape[1]), np.float64)
    cnt = np.zeros(n_dst)
    for s, t in edges.T:
        out[t] += src[s]
        cnt[t] += 1
    return out / np.maximum(cnt, 1)[:, None]


def test_files_layout(tmp_path):
    from dgraph_amd.data.mag240m import MAG240MFiles

    make_fake_mag(str(tmp_path))
    f = MAG240MFiles(str(tmp_path))
    assert (f.num_papers, f.num_authors, f.num_institutions) == (NP, NA, NI)
    assert f.paper_feat.shape == (NP, F) and isinstance(f.paper_feat, np.memmap)
    assert np.array_equal(f.edge_index("author", "institution"),
                          f.edge_index("author", "affiliated_with", "institution"))
    assert np.array_equal(f.edge_index("author", "paper"),
                          f.edge_index("author", "writes", "paper"))
    assert len(f.get_idx_split("train")) == 30 and f.num_classes == 153


def test_derived_features_match_numpy_mean(tmp_path):
    from dgraph_amd.data.mag240m import MAG240MFiles, generate_feature_data

    make_fake_mag(str(tmp_path))
    f = MAG240MFiles(str(tmp_path))
    paths = generate_feature_data(f, None, device=torch.device("cpu"))
    af = np.load(paths["author"])
    inst = np.load(paths["institution"])
    w = np.asarray(f.edge_index("author", "writes", "paper"))
    a = np.asarray(f.edge_index("author", "affiliated_with", "institution"))
    ref_a = _np_mean(np.asarray(f.paper_feat, np.float64), w[::-1], NA)
    ref_i = _np_mean(af.astype(np.float64), a, NI)
    np.testing.assert_allclose(af, ref_a, atol=2e-3, rtol=2e-3)
    np.testing.assert_allclose(inst, ref_i, atol=2e-3, rtol=2e-3)
    assert af.dtype == np.float16 and af.shape == (NA, F)


class _Comm:
    def __init__(self, rank=0, world=1, group=None):
        self.r, self.w, self.group = rank, world, group

    def get_rank(self):
        return self.r

    def get_world_size(self):
        return self.w

    def barrier(self):
        if self.w > 1:
            import torch.distributed as dist
            dist.barrier()


def test_dataset_single_rank_and_plan_cache(tmp_path, monkeypatch):
    from dgraph_amd.data import mag240m

    d = make_fake_mag(str(tmp_path))
    ds = mag240m.DGraph_MAG240M_Dataset(_Comm(), data_dir=d, real_features=True)
    assert os.path.exists(os.path.join(d, "MAG240M_dataset_rank_0_of_1_comm_plans.pt"))
    assert [x.shape for x in ds.features] == [(NP, F), (NA, F), (NI, F)]
    assert ds.num_relations == 5 and ds.num_classes == 153
    assert int(ds.relations[0].csr.nnz) == 2 * np.load(
        os.path.join(d, "processed/paper___cites___paper/edge_index.npy")).shape[1]
    assert ds.get_mask("train").numel() == 30
    # the second construction must come from the plan file
    monkeypatch.setattr(mag240m, "build_relation_graph",
                        lambda *a, **k: (_ for _ in ()).throw(AssertionError("rebuilt")))
    ds2 = mag240m.DGraph_MAG240M_Dataset(_Comm(), data_dir=d)
    for a, b in zip(ds.relations, ds2.relations):
        assert torch.equal(a.csr.rowptr, b.csr.rowptr) and torch.equal(a.csr.col, b.csr.col)
    assert ds2.features[0].shape == (NP, 1)  # reference setting: randn(n, 1)
    assert ds2.paper_2_author_comm_plan is ds2.relations[1]


def test_rank_mapping_must_be_sorted(tmp_path):
    from dgraph_amd.data.mag240m import DGraph_MAG240M_Dataset

    d = make_fake_mag(str(tmp_path))
    with pytest.raises(ValueError):
        DGraph_MAG240M_Dataset(_Comm(), data_dir=d,
                               paper_rank_mappings=torch.arange(NP) % 2)


def _mag_dist(rank, world, d):
    from dgraph_amd.data.mag240m import DGraph_MAG240M_Dataset

    ds = DGraph_MAG240M_Dataset(_Comm(rank, world), data_dir=d, real_features=True)
    lo = int(ds.offsets[1][rank])
    af = np.load(os.path.join(d, "author_feat.npy"))
    assert torch.equal(ds.features[1], torch.from_numpy(af[lo:lo + ds.features[1].shape[0]]).float())
    assert os.path.exists(os.path.join(d, f"MAG240M_dataset_rank_{rank}_of_{world}_comm_plans.pt"))
    import torch.distributed as dist
    nnz = torch.tensor([int(r.csr.nnz) for r in ds.relations])
    dist.all_reduce(nnz)
    w = np.load(os.path.join(d, "processed/author___writes___paper/edge_index.npy"))
    assert int(nnz[1]) == w.shape[1] and int(nnz[2]) == w.shape[1]


@pytest.mark.parametrize("world", [2, 4])
def test_dataset_distributed(tmp_path, ranks, world):
    d = make_fake_mag(str(tmp_path))
    ranks(_mag_dist, world, d)


def test_stale_plan_file_is_rebuilt(tmp_path):
    from dgraph_amd.data import mag240m

    d = make_fake_mag(str(tmp_path))
    mag240m.DGraph_MAG240M_Dataset(_Comm(), data_dir=d)
    path = os.path.join(d, "MAG240M_dataset_rank_0_of_1_comm_plans.pt")
    blob = torch.load(path, weights_only=True)
    blob["_meta"][0] += 1  # pretend it was written for another graph
    torch.save(blob, path)
    with pytest.raises(ValueError):
        mag240m.DGraph_MAG240M_Dataset(_Comm(), data_dir=d, cached_comm_plans=path)
    ds = mag240m.DGraph_MAG240M_Dataset(_Comm(), data_dir=d)  # default path: rebuilt
    assert torch.equal(torch.load(path, weights_only=True)["_meta"][:3],
                       torch.tensor([NP, NA, NI]))
    assert ds.num_relations == 5
