"""The memory-lean fp32 executor (models/sage_fused.py) against the layer-stack autograd
path of the same GraphSAGE: loss, every weight gradient and the validation/test hits, on
one rank (CPU reference kernels) and vertex-partitioned over W = 2 / 4 gloo ranks
(all-reduced gradients equal the W=1 gradients)."""
import pytest
import torch
import torch.distributed as dist

from dgraph_amd.data.synthetic import (SHAPES, SPLIT_TEST, SPLIT_TRAIN, SPLIT_VALID,
                                       build_partition, contiguous_offsets, node_data)
from dgraph_amd.models.sage import GraphSAGE
from dgraph_amd.models.sage_fused import FusedSAGE
from dgraph_amd.parallel.dist_graph import DistGraph

SCALE = 2e-5  # ~2.2K vertices, ~65K messages


def _setup(rank, world, dev="cpu", layers=3, chunk_rows=300, gf=0.3, name="ogbn-papers100M",
           hidden=256):
    # ogbn-products: 100 input features (zero-padded to 128 inside the executor), 47 classes
    shape = SHAPES[name].scaled(SCALE if name == "ogbn-papers100M" else 1e-3)
    part = build_partition(shape, rank, world, dev, global_frac=gf, window=64)
    csr = part["csr"]
    if world == 1:
        csr.num_cols = part["L"]
    group = dist.group.WORLD if world > 1 else None
    g = DistGraph(csr, part["L"], part["H"], part["send_local_idx"], part["send_splits"],
                  part["recv_splits"], group, symmetric=True)
    offs = contiguous_offsets(shape.num_nodes, world)
    x, y, split = node_data(shape, rank, offs, dev, dtype=torch.float32, return_split=True)
    tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
    ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
    n_tr = torch.tensor([tr.numel()])
    if world > 1:
        dist.all_reduce(n_tr)
    # products, seed 0: a layer-2 pre-activation of 6e-8 (a ReLU tie that summation order
    # flips) — seed 1 keeps every |pre-activation| well above fp32 rounding
    torch.manual_seed(0 if name == "ogbn-papers100M" else 1)
    model = GraphSAGE(shape.num_features, hidden, shape.num_classes, layers).to(dev)
    return shape, g, x, y, split, tr, ev, int(n_tr), model


def _fused_grads(rank, world, layers=3, chunk_rows=300, name="ogbn-papers100M",
                 schedule="full", dev="cpu", gf=0.3, hidden=256, **knobs):
    """schedule (W > 1): "full" = forward exchanges overlapped through the whole-layer
    aggregate buffer (output layer) and in place (hidden layers); "inplace" = no whole-layer
    buffer (hidden layers in place, the output layer's exchange waited for up front);
    "off" = every exchange waited for up front."""
    from dgraph_amd.utils.config import ExecutorConfig

    shape, g, x, y, split, tr, ev, n_tr, model = _setup(rank, world, dev=dev, layers=layers,
                                                        name=name, gf=gf, hidden=hidden)
    cfg = ExecutorConfig(overlap=schedule != "off", **knobs)
    ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID, n_tr,
                   chunk_rows=chunk_rows, config=cfg)
    if schedule == "inplace":
        ex.agg_full = None
    if world > 1:
        assert (ex.agg_full is not None) == (schedule == "full")
    loss = ex.step()
    grads = [p.grad.clone() for p in model.parameters()]
    return loss, grads, ex.correct.clone()


@pytest.mark.parametrize("world", [1, 2])
def test_compact_transposed_adjacency_matches_column_map(ranks, world, tmp_path):
    """The input-layer backward over the S-compacted transposed adjacency (COMPACT_T) and
    over the column-mapped full adjacency give the same step."""
    if world == 1:
        res = {}
        for mode in ("on", "off"):
            res[mode] = _fused_grads(0, 1, compact_t=mode)
        (l1, g1, c1), (l2, g2, c2) = res["on"], res["off"]
        torch.testing.assert_close(l1, l2)
        for a, b in zip(g1, g2):
            torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
        assert torch.equal(c1, c2)
    else:
        ranks(_compact_body, world, str(tmp_path / "r.pt"))


def _compact_body(rank, world, path):
    import torch.distributed as dist

    out = {}
    for mode in ("on", "off"):
        loss, grads, corr = _fused_grads(rank, world, schedule="off", compact_t=mode)
        for t in grads:
            dist.all_reduce(t)
        out[mode] = (loss, grads)
    for a, b in zip(out["on"][1], out["off"][1]):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)


def _stack_grads(layers=3, name="ogbn-papers100M"):
    shape, g, x, y, split, tr, ev, n_tr, model = _setup(0, 1, layers=layers, name=name)
    logits, evl = model(x, g, out_rows=tr, eval_rows=ev)
    loss = torch.nn.functional.cross_entropy(logits.float(), y[tr], reduction="sum") / n_tr
    loss.backward()
    hit = evl.argmax(1) == y[ev]
    iv = split[ev] == SPLIT_VALID
    corr = torch.tensor([(hit & iv).sum(), (hit & ~iv).sum()])
    return loss.detach(), [p.grad.clone() for p in model.parameters()], corr


@pytest.mark.parametrize("layers,name", [(2, "ogbn-papers100M"), (3, "ogbn-papers100M"),
                                         (2, "ogbn-products"), (3, "ogbn-products")])
def test_fused_matches_stack_w1(layers, name):
    l0, g0, c0 = _stack_grads(layers, name)
    l1, g1, c1 = _fused_grads(0, 1, layers, name=name)
    torch.testing.assert_close(l1, l0, atol=1e-5, rtol=1e-5)
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-4)
    assert torch.equal(c1, c0)


def _dist_body(rank, world, ref_path, schedule="full"):
    loss, grads, corr = _fused_grads(rank, world, schedule=schedule)
    for t in grads:
        dist.all_reduce(t)
    dist.all_reduce(loss)
    dist.all_reduce(corr)
    ref = torch.load(ref_path)
    torch.testing.assert_close(loss, ref["loss"], atol=1e-5, rtol=1e-5)
    for a, b in zip(grads, ref["grads"]):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-4)
    assert torch.equal(corr, ref["corr"])


@pytest.mark.parametrize("world,schedule", [(2, "full"), (4, "full"), (2, "inplace"),
                                            (2, "off")])
def test_fused_partitioned_matches_w1(ranks, world, schedule, tmp_path):
    loss, grads, corr = _fused_grads(0, 1)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_dist_body, world, str(p), schedule)


def _directed(csr, L, seed=0):
    """Drop ~30 % of the entries of a symmetric local CSR: a directed graph (A != A^T)."""
    from dgraph_amd.ops.csr import CSR

    g = torch.Generator().manual_seed(seed)
    keep = torch.rand(csr.col.numel(), generator=g) > 0.3
    rows = csr.row_ids()[keep]
    cols = csr.col[keep]
    return CSR.from_coo(rows, cols, L, csr.num_cols, keep_perm=False)


def test_fused_directed_graph_matches_autograd():
    """on a non-symmetric graph B1b must aggregate over A^T, not A's own rows.
    The fused executor equals the layer-stack autograd path on a directed graph."""
    shape = SHAPES["ogbn-papers100M"].scaled(SCALE)
    part = build_partition(shape, 0, 1, "cpu", global_frac=0.3, window=64)
    L = part["L"]
    part["csr"].num_cols = L
    csr = _directed(part["csr"], L)
    assert not torch.equal(csr.col, part["csr"].col)
    offs = contiguous_offsets(shape.num_nodes, 1)
    x, y, split = node_data(shape, 0, offs, "cpu", dtype=torch.float32, return_split=True)
    tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
    ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
    res = []
    for fused in (False, True):
        g = DistGraph(csr, L, 0, symmetric=False)
        torch.manual_seed(0)
        model = GraphSAGE(shape.num_features, 256, shape.num_classes, 3)
        if fused:
            ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID,
                           tr.numel(), chunk_rows=300)
            assert ex.itT is not None
            loss = ex.step()
        else:
            logits, _ = model(x, g, out_rows=tr, eval_rows=ev)
            loss = torch.nn.functional.cross_entropy(logits.float(), y[tr],
                                                     reduction="sum") / tr.numel()
            loss.backward()
        res.append((loss.detach(), [p.grad.clone() for p in model.parameters()]))
    torch.testing.assert_close(res[1][0], res[0][0], atol=1e-5, rtol=1e-5)
    for a, b in zip(res[1][1], res[0][1]):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-4)


def _interior_first_body(rank, world, ref_path, overlap, store="auto", stream="off",
                         keep_as="auto", hidden=256, bwd_halo="pull", pf="auto"):
    """One rank of a W-way partition renumbered interior-first (parallel/reorder.py), the
    fused executor's interior-then-boundary schedule, all-reduced against W=1."""
    from dgraph_amd.parallel.reorder import interior_first
    from dgraph_amd.utils.config import ExecutorConfig

    cfg = ExecutorConfig(overlap=overlap, boundary_store=store, keep_as=keep_as,
                         bwd_halo=bwd_halo, project_first=pf,
                         halo_stream="on" if stream != "off" else "off")
    if stream == "single":  # one ring buffer: exchange and aggregation alternate
        cfg.stream_shapes = "64x1"
    if stream == "ramp":  # half-width first block, output-layer self term as the fill
        cfg.stream_ramp = cfg.stream_out_fill = True
        cfg.project_first = "off"  # (the self-term fill is the aggregate-first output layer's)
    if stream != "off":  # the input's static halo exchanged in 16-column blocks too
        DistGraph.STATIC_BLOCK_BYTES = 1024
    shape = SHAPES["ogbn-papers100M"].scaled(SCALE)
    part = build_partition(shape, rank, world, "cpu", global_frac=0.05, window=64)
    csr, send, perm, L_int, loc = interior_first(part["csr"], part["L"],
                                                 part["send_local_idx"])
    assert 0 < L_int < part["L"]
    g = DistGraph(csr, part["L"], part["H"], send, part["send_splits"], part["recv_splits"],
                  dist.group.WORLD, symmetric=True)
    offs = contiguous_offsets(shape.num_nodes, world)
    x, y, split = node_data(shape, rank, offs, "cpu", dtype=torch.float32, return_split=True)
    x, y, split = x[perm], y[perm], split[perm]
    tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
    ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
    n_tr = torch.tensor([tr.numel()])
    dist.all_reduce(n_tr)
    torch.manual_seed(0)
    model = GraphSAGE(shape.num_features, hidden, shape.num_classes, 3)
    ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID, int(n_tr),
                   chunk_rows=300, release_graph=True, config=cfg)
    assert ex.Li == L_int and ex.nA >= 1
    assert (ex.aS_keep is not None) == (keep_as != "off" or stream != "off")
    if store != "auto":
        assert ex.use_store == {"hidden": store == "on", "out": store == "on"}
    assert ex.stream == (stream != "off")
    # the output layer projected before its aggregation (Cp 176 < hidden): on by plan
    assert (ex.pf is not None) == (stream != "ramp" and pf != "off")
    # the input layer's backward halo: pulled S rows of u (symmetric graph), else pushed
    assert (ex.pull is not None) == (bwd_halo == "pull")
    if ex.pull is not None:
        assert 0 < ex.pull["n_send"] < ex.n_send and ex.pull["n_recv"] < ex.H
    # streamed pulls run B1b over the compacted, pre-mapped adjacency (compact_pull=auto)
    assert (ex.PT is not None) == (ex.stream and ex.pull is not None)
    if stream == "single":
        assert ex.nbuf == 1
    if stream == "ramp":
        assert ex.zself is not None and len(ex._stream_blocks(256)) == 5
    assert g.interior is None  # released: the executor runs on its own adjacency
    loss = ex.step()
    grads = [p.grad.clone() for p in model.parameters()]
    corr = ex.correct.clone()
    for t in grads:
        dist.all_reduce(t)
    dist.all_reduce(loss)
    dist.all_reduce(corr)
    ref = torch.load(ref_path)
    torch.testing.assert_close(loss, ref["loss"], atol=1e-5, rtol=1e-5)
    for a, b in zip(grads, ref["grads"]):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-4)
    assert torch.equal(corr, ref["corr"])


@pytest.mark.parametrize("world,overlap,store,stream", [
    (2, True, "on", "off"), (2, True, "off", "off"), (4, True, "on", "off"),
    (4, True, "off", "off"), (2, False, "auto", "off"),
    # streamed halos (column blocks through a buffer ring; the structureless-graph plan)
    (2, True, "auto", "on"), (4, True, "auto", "on"), (8, True, "auto", "on"),
    (2, True, "auto", "single"), (2, True, "auto", "ramp")])
def test_fused_interior_first_matches_w1(ranks, world, overlap, store, stream, tmp_path):
    loss, grads, corr = _fused_grads(0, 1, gf=0.05)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_interior_first_body, world, str(p), overlap, store, stream)


@pytest.mark.parametrize("world,stream", [(2, "off"), (4, "off"), (2, "on")])
def test_fused_bwd_halo_push_matches_w1(ranks, world, stream, tmp_path):
    """The input layer's backward halo by "push" (contributions to every halo row sent back
    to the owners, the non-symmetric graphs' path) instead of the default "pull", resident
    and streamed."""
    loss, grads, corr = _fused_grads(0, 1, gf=0.05)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_interior_first_body, world, str(p), True, "auto", stream, "auto", 256, "push")


@pytest.mark.parametrize("world,stream", [(2, "off"), (4, "on")])
def test_fused_aggregate_first_output_matches_w1(ranks, world, stream, tmp_path):
    """The output layer aggregated before its projection at W > 1 (PROJECT_FIRST=off, the
    W=1 order) instead of projected first."""
    loss, grads, corr = _fused_grads(0, 1, gf=0.05)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_interior_first_body, world, str(p), True, "auto", stream, "auto", 256, "pull",
          "off")


@pytest.mark.parametrize("world,store,stream,keep_as", [
    (2, "on", "off", "off"),   # S rows re-aggregated in the backward (resident halo)
    (2, "auto", "on", "on"),   # S-row aggregate kept from the streamed forward
    (4, "off", "off", "on")])
def test_fused_keep_support_aggregate(ranks, world, store, stream, keep_as, tmp_path):
    """The last hidden layer's input aggregate on the support rows kept from the forward
    (or recomputed in the backward): same gradients as W=1."""
    loss, grads, corr = _fused_grads(0, 1, gf=0.05)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_interior_first_body, world, str(p), True, store, stream, keep_as)


def test_fused_hidden512_store_stream_matches_w1(ranks, tmp_path):
    """a 512-wide hidden layer with the boundary-row store and with streamed
    halos (the in-place aggregate-then-GEMM paths at N > 256) at W=2."""
    loss, grads, corr = _fused_grads(0, 1, gf=0.05, hidden=512)
    p = tmp_path / "ref.pt"
    torch.save({"loss": loss, "grads": grads, "corr": corr}, p)
    ranks(_interior_first_body, 2, str(p), True, "on", "off", "auto", 512)
    ranks(_interior_first_body, 2, str(p), True, "auto", "on", "auto", 512)


@pytest.mark.parametrize("hidden,feat", [(128, 100), (512, 128), (256, 300)])
def test_fused_widths_match_stack(hidden, feat):
    """Hidden 128 / 512 and a wide (zero-padded) input run on the fused executor and equal
    the layer-stack autograd path."""
    from dgraph_amd.data.synthetic import GraphShape

    base = SHAPES["ogbn-papers100M"].scaled(SCALE)
    shape = GraphShape("w", base.num_nodes, base.num_directed_edges, feat, 40, 0.3, 0.1, 0.1)
    part = build_partition(shape, 0, 1, "cpu", global_frac=0.3, window=64)
    L = part["L"]
    part["csr"].num_cols = L
    offs = contiguous_offsets(shape.num_nodes, 1)
    x, y, split = node_data(shape, 0, offs, "cpu", dtype=torch.float32, return_split=True)
    tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
    ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
    res = []
    for fused in (False, True):
        g = DistGraph(part["csr"], L, 0, symmetric=True)
        torch.manual_seed(0)
        model = GraphSAGE(feat, hidden, 40, 3)
        if fused:
            from dgraph_amd.models.sage_fused import supported

            assert supported(model, x)
            ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID,
                           tr.numel(), chunk_rows=300)
            loss = ex.step()
        else:
            logits, _ = model(x, g, out_rows=tr, eval_rows=ev)
            loss = torch.nn.functional.cross_entropy(logits.float(), y[tr],
                                                     reduction="sum") / tr.numel()
            loss.backward()
        res.append((loss.detach(), [p.grad.clone() for p in model.parameters()]))
    torch.testing.assert_close(res[1][0], res[0][0], atol=1e-5, rtol=1e-5)
    for a, b in zip(res[1][1], res[0][1]):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-4)


def test_executor_config_resolved_at_construction(monkeypatch):
    """The schedule knobs are read when an executor is BUILT (they were module
    globals frozen at import): an environment change after import changes the next
    executor's schedule, and an explicit config wins over the environment."""
    from dgraph_amd.utils.config import ExecutorConfig, RunConfig

    shape, g, x, y, split, tr, ev, n_tr, model = _setup(0, 1)

    def build(**kw):
        return FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID, n_tr,
                         chunk_rows=300, **kw)

    monkeypatch.setenv("DGRAPH_FUSED_KEEP_AGG0", "off")
    a = build()
    assert a.cfg.keep_agg0 == "off" and a.schedule["keep_agg0"] is False
    monkeypatch.setenv("DGRAPH_FUSED_KEEP_AGG0", "on")
    b = build()
    assert b.schedule["keep_agg0"] is True
    c = build(config=ExecutorConfig(keep_agg0="off"))
    assert c.schedule["keep_agg0"] is False
    # the same knobs through the run config (bench.py records cfg.to_dict() whole)
    monkeypatch.setenv("DGRAPH_FUSED_HALO_STREAM", "on")
    monkeypatch.setenv("DGRAPH_PLAN_LINK_GBPS", "75")
    rc = RunConfig.from_env()
    assert rc.fused.halo_stream == "on" and rc.fused.plan_link_gbps == 75.0
    assert rc.to_dict()["fused"]["keep_agg0"] == "on"
    assert rc.model.dtype == "fp32"
    with pytest.raises(ValueError):
        ExecutorConfig(halo_stream="sometimes")


def test_memory_plan_recorded():
    """The setup's memory plan lists each optional buffer with its bytes, the room it was
    decided against and whether it was taken; the recorded choices are the executor's."""
    shape, g, x, y, split, tr, ev, n_tr, model = _setup(0, 1)
    ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID, n_tr,
                   chunk_rows=300)
    plan = ex.schedule["memory_plan"]
    by = {m["what"]: m for m in plan}
    assert {"keep_aS", "keep_agg0", "chunk_arena"} <= set(by)
    assert by["keep_agg0"]["taken"] == (ex.agg0 is not None)
    assert by["keep_aS"]["taken"] == (ex.aS_keep is not None)
    assert by["chunk_arena"]["gb"] >= 0 and all(m["room_gb"] >= 0 for m in plan)
    # room only shrinks as buffers are taken
    rooms = [m["room_gb"] for m in plan]
    assert rooms == sorted(rooms, reverse=True)
