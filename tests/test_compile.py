"""torch.compile(model, dynamic=True) — the reference's `compile=True` path (gin.py:56,
gat.py:84, drgnet.py:103; configs/config.py:64) — traced on CPU with meta tensors.

Every HIP op is a torch.library custom op with a fake kernel (lesion_gnn_amd/library.py), so
Dynamo traces each model in ONE graph (fullgraph=True: no graph break) with symbolic sizes, and
AOTAutograd derives the backward graph from the ops' registered autograd formulas. The fake
kernels run on meta tensors here (shape propagation only — nothing launches); the GPU test
tests/test_gpu_compile.py runs the same compiled models on the HIP kernels against the oracle.
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import synth
from lesion_gnn_amd.models import DRGNet, GAT, GCN, GIN

# what may appear besides lgnn:: ops: tuple unpacking of list outputs, the 0-element placeholder
# of an absent tensor, autograd bookkeeping, and the functionalized running-stat update
GLUE = {"<built-in function getitem>", "aten.empty.memory_format", "aten.detach.default",
        "auto_functionalized_v2", "auto_functionalized"}
# views of one op output (offsets are symbolic-size arithmetic; views launch nothing)
VIEWS = {"aten.slice.Tensor", "aten.view.default", "aten.split_with_sizes.default",
         "<built-in function add>",
         "<built-in function floordiv>", "<built-in function mul>"}


def trace(model, args):
    seen = []

    def backend(gm, example_inputs):
        from functorch.compile import make_boxed_func
        from torch._functorch.aot_autograd import aot_module_simplified

        def grab(g, _inputs):
            seen.append({str(n.target) for n in g.graph.nodes if n.op == "call_function"})
            return make_boxed_func(g)

        return aot_module_simplified(gm, example_inputs, fw_compiler=grab, bw_compiler=grab)

    torch._dynamo.reset()
    cm = torch.compile(model, backend=backend, fullgraph=True, dynamic=True)
    out = cm(*args)
    out.float().sum().backward()
    assert len(seen) == 2  # one forward and one backward graph
    return out, seen[0], seen[1]


def meta_args(b, *extra):
    return (b.x.to("meta"), b.edge_index.to("meta"), b.batch.to("meta"), *extra, b.num_graphs)


@pytest.mark.parametrize("name", ["gat_c3_bf16", "gat_fp32", "gat_refcfg_dropout", "gin_train",
                                  "gin_eval", "gin_dropout", "gcn", "gcn_dropout"])
def test_models_trace_to_lgnn_ops_only(name):
    """Dropout included (the reference config trains with dropout 0.35, configs/config.py:63):
    its masks come from lgnn::dropout_masks and the between-conv product is lgnn::mask_mul, so no
    aten random / elementwise op (nothing for Inductor to generate) appears in either graph."""
    torch.manual_seed(0)
    drop = "dropout" in name
    if name.startswith("gat"):
        d_in = 1025 if ("c3" in name or "refcfg" in name) else 128
        b = synth.make_batch(6, n=20, k=6, d_in=d_in, seed=1, sizes="lognormal")
        heads = 2 if "refcfg" in name else 4
        m = GAT(d_in, [128] * 4, 1, heads=heads, dropout=0.35 if drop else 0.0,
                precision="bf16" if "bf16" in name else "fp32").train()
        want = {"lgnn.gat_conv.default", "lgnn.graph_build_b.default",
                "lgnn.gat_conv_head.default"}
    elif name.startswith("gin"):
        b = synth.make_batch(6, n=64, k=8, d_in=128, seed=2)
        m = GIN(128, [128, 128, 128], 5, 0.35 if drop else 0.0, pool="add")
        m.train(name != "gin_eval")
        want = {"lgnn.gin_conv.default", "lgnn.node_linear.default"}
        if name != "gin_eval":
            want.add("auto_functionalized_v2")  # the BN running-stat update (mutating op)
        if drop:
            want.add("lgnn.mask_mul.default")
    else:
        b = synth.make_batch(6, n=64, k=8, d_in=128, seed=3)
        m = GCN(128, [128, 128, 128], 5, 0.1 if drop else 0.0).train()
        want = {"lgnn.node_linear.default", "lgnn.mask_mul.default"} if drop \
            else {"lgnn.gcn_stack.default"}
    out, fw, bw = trace(m.to("meta"), meta_args(b))
    assert out.shape[0] == b.num_graphs
    # views launch nothing (the dropout masks are views of one op output; GAT's attention / bias
    # gradients views of one reduction buffer)
    extra = {t for t in (fw | bw) - GLUE - VIEWS if not t.startswith("<function sym_")}
    if drop:  # the generator state's counter advance is the op's declared mutation
        assert "auto_functionalized_v2" in fw or "lgnn.dropout_masks.default" in fw, sorted(fw)
    assert all(t.startswith("lgnn.") for t in extra), sorted(extra)
    assert want <= fw | bw, (want, sorted(fw | bw))
    assert any(t.endswith("_bwd.default") for t in bw), sorted(bw)


def test_drgnet_traces_in_one_graph():
    """DRGNet: the GraphConv stack, the weighted CSR and SortAggregation are lgnn ops; the head
    (Conv1d / MaxPool1d / Linear / ELU, drgnet.py:41-48,62-67) stays torch's, as in the
    reference."""
    b = synth.make_batch(6, n=24, k=6, d_in=16, seed=4, sizes="lognormal")
    ew = ref.gaussian_distance(b.edge_index, b.pos, 0.1).float()
    m = DRGNet(16, 8, 2, 10, 5).eval().to("meta")
    out, fw, bw = trace(m, meta_args(b, ew.to("meta")))
    assert out.shape == (6, 5)
    for op in ("lgnn.sort_pool.default", "lgnn.spmm.default", "lgnn.weighted_csr.default"):
        assert op in fw, op
    assert "lgnn.graph_build_b.default" in fw or "lgnn.graph_build.default" in fw
    assert "lgnn.sort_pool_bwd.default" in bw


def test_config_compile_flag_wraps_model():
    from lesion_gnn_amd.models import GATConfig, OptimizerConfig, get_model

    cfg = GATConfig(hiddden_channels=[32, 32], heads=2, dropout=0.0, compile=True,
                    optimizer=OptimizerConfig(loss_type="MSE"))
    cfg.input_features.value = 8
    cfg.num_classes.value = 5
    module = get_model(cfg)
    assert isinstance(module.model, torch._dynamo.eval_frame.OptimizedModule)
    cfg.compile = False
    assert isinstance(get_model(cfg).model, GAT)


def test_weight_bundle_sizes_match_the_library():
    """ops._s3_bundle_sizes (the Python restatement Dynamo traces) == lgnn_s3_weight_planes_numel
    for every shape class: K % 64 != 0, N > 128, transposed, 1 and 3 planes."""
    from lesion_gnn_amd import _lib, ops

    lib = _lib.load()
    for rows, cols in [(128, 1025), (128, 128), (256, 128), (300, 37), (5, 3), (512, 512)]:
        for t in (False, True):
            for bf16 in (False, True):
                o, i = (cols, rows) if t else (rows, cols)
                want = lib.lgnn_s3_weight_planes_numel(o, i, 1 if bf16 else 3)
                assert ops._s3_bundle_sizes([(rows, cols)], [t], bf16) == [want]
