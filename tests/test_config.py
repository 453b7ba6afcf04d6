"""CPU checks of the config / registry surface (reference models/__init__.py:10,22-35,
configs/config.py:59-65, utils/placeholder.py): the experiment's model section builds against
this package's classes unchanged (field names incl. the `hiddden_channels` typo), Placeholder
semantics, isinstance dispatch, and state_dict keys identical to the PyG-named oracle modules."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd.models import (GATConfig, GCNConfig, GINConfig, LossType, OptimizerAlgo,
                                   OptimizerConfig, get_model)
from lesion_gnn_amd.models.gat import GATModule
from lesion_gnn_amd.models.gin import GINModule
from lesion_gnn_amd.utils import ClassWeights, Placeholder


def reference_model_section():
    """The `model=` block of reference configs/config.py:56-65, verbatim field values."""
    return GATConfig(
        optimizer=OptimizerConfig(
            lr=1e-3,
            lr_scheduler=None,
            weight_decay=2e-6,
            algo=OptimizerAlgo.ADAM,
            loss_type=LossType.MSE,
            class_weights_mode=ClassWeights.UNIFORM,
        ),
        hiddden_channels=[128] * 4,
        heads=2,
        dropout=0.35,
        compile=True,
    )


def test_reference_config_builds_gat():
    cfg = reference_model_section()
    cfg.num_classes.value = 5          # training.py:23-27 fills the placeholders
    cfg.input_features.value = 1025
    cfg.optimizer.class_weights.value = torch.ones(5)
    m = get_model(cfg)
    assert isinstance(m, GATModule) and m.is_regression
    assert m.model.out_proj.out_features == 1  # regression -> 1 output (gat.py:79)
    assert len(m.model.convs) == 3 and m.model.convs[0].heads == 2
    opt = m.configure_optimizers()
    from lesion_gnn_amd import optim
    assert isinstance(opt, optim.Adam) and isinstance(opt, torch.optim.Optimizer)
    want = ref.GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).state_dict()
    # compile=True: the model is torch.compile'd as in the reference (gat.py:84), so its keys
    # carry the `_orig_mod.` prefix exactly as the reference's compiled module's do
    assert {k: v.shape for k, v in m.model.state_dict().items()} == \
        {"_orig_mod." + k: v.shape for k, v in want.items()}


def test_gin_and_gcn_configs():
    gin = GINConfig(optimizer=OptimizerConfig(), hidden_channels=[128, 128, 128], dropout=0.0,
                    compile=False, pool="add")
    gin.num_classes.value, gin.input_features.value = 5, 128
    with pytest.raises(ValueError):  # CE reads the class-weights placeholder (base.py:93-94)
        get_model(gin)
    gin.optimizer.class_weights.value = torch.ones(5)
    m = get_model(gin)
    assert isinstance(m, GINModule) and m.model.pool == "add"
    want = ref.GIN(128, [128, 128, 128], 5, 0.0).state_dict()
    assert {k: v.shape for k, v in m.model.state_dict().items()} == \
        {k: v.shape for k, v in want.items()}
    gcn = GCNConfig(optimizer=OptimizerConfig(), hidden_channels=[64, 64], dropout=0.1,
                    compile=False)
    gcn.num_classes.value, gcn.input_features.value = 3, 32
    gcn.optimizer.class_weights.value = torch.ones(3)
    assert get_model(gcn).model.convs[0].lin.weight.shape == (64, 64)


def test_placeholder_and_unknown_config():
    p = Placeholder()
    with pytest.raises(ValueError):
        _ = p.value
    p.value = 3
    assert p.value == 3
    with pytest.raises(ValueError):
        get_model(object())


def test_gat_settransformer_readout_out_of_scope():
    from lesion_gnn_amd.models.gat import GAT

    with pytest.raises(NotImplementedError):
        GAT(8, [8, 8], 2, heads=2, dropout=0.0, num_st_seed_points=4)


REFERENCE_CONFIG = "/root/reference/configs/config.py"

EXPERIMENT = '''
from lesion_gnn.datasets.aptos import AptosConfig
from lesion_gnn.datasets.datamodule import DataConfig
from lesion_gnn.datasets.ddr import DDRConfig, DDRVariant
from lesion_gnn.datasets.nodes.lesions import LesionsNodesConfig, TimmEncoderFeatures
from lesion_gnn.models.base import LossType, OptimizerAlgo, OptimizerConfig
from lesion_gnn.models.gin import GINConfig
from lesion_gnn.transforms import TransformConfig
from lesion_gnn.utils import ClassWeights
from lesion_gnn.utils.config import Config

NODES = LesionsNodesConfig(feature_source=TimmEncoderFeatures(timm_model="m", layer=-1))
cfg = Config(
    dataset=DataConfig(
        train_datasets=[DDRConfig(root="d", nodes=NODES, variant=DDRVariant.TRAIN)],
        val_datasets=[DDRConfig(root="d", nodes=NODES, variant=DDRVariant.VALID)],
        test_datasets=[AptosConfig(root="a", nodes=NODES)],
        transforms=[TransformConfig(name="KNNGraph", kwargs={"k": 8, "loop": True}),
                    TransformConfig(name="GaussianDistance", kwargs={"sigma": 0.5})],
        batch_size=64, num_workers=0),
    model=GINConfig(optimizer=OptimizerConfig(lr=1e-3, algo=OptimizerAlgo.ADAMW,
                                              loss_type=LossType.CE,
                                              class_weights_mode=ClassWeights.INVERSE),
                    hidden_channels=[64, 64, 64], dropout=0.1, compile=False),
    monitored_metric="val_DDR_kappa", monitor_mode="max", max_epochs=3, seed=7,
    project_name="p", tags=["T"])
'''


def _fill_and_build(cfg, classes=5, d_in=1025):
    """training.py:23-27: fill the placeholders from the dataset, then get_model (:31)."""
    cfg.model.num_classes.value = classes
    cfg.model.input_features.value = d_in
    cfg.model.optimizer.class_weights.value = torch.ones(classes)
    return get_model(cfg.model)


def test_experiment_file_with_reference_imports(tmp_path):
    """A Python experiment file written against the reference's module paths (lesion_gnn.*)
    loads through utils.config.get_config and yields this package's classes."""
    from lesion_gnn_amd.datasets.datamodule import compose_transforms
    from lesion_gnn_amd.knn import KNNGraph
    from lesion_gnn_amd.transforms import GaussianDistance
    from lesion_gnn_amd.utils.config import Config, get_config

    f = tmp_path / "exp.py"
    f.write_text(EXPERIMENT)
    cfg = get_config(f, module_name="exp_cfg_test")
    assert isinstance(cfg, Config) and isinstance(cfg.model, GINConfig)
    assert cfg.dataset.train_datasets[0].name == "DDR"
    assert cfg.dataset.test_datasets[0].name == "Aptos"
    m = _fill_and_build(cfg, d_in=128)
    assert isinstance(m, GINModule) and len(m.model.convs) == 2
    t = compose_transforms(cfg.dataset, compile=cfg.model.compile)
    assert isinstance(t.transforms[0], KNNGraph) and t.transforms[0].k == 8
    assert isinstance(t.transforms[1], GaussianDistance) and t.transforms[1].sigma == 0.5
    assert repr(t.transforms[-1]) == "ToSparseTensor()"  # compile=False (datamodule.py:44-45)


@pytest.mark.skipif(not __import__("os").path.exists(REFERENCE_CONFIG),
                    reason="reference checkout not mounted (GPU box)")
def test_reference_config_file_loads_unchanged():
    """The reference's own experiment file, read in place (not copied), builds against this
    package: GAT with hiddden_channels=[128]*4, heads 2, MSE (configs/config.py:56-65)."""
    from lesion_gnn_amd.utils.config import Config, get_config

    cfg = get_config(REFERENCE_CONFIG)
    assert isinstance(cfg, Config) and isinstance(cfg.model, GATConfig)
    assert cfg.model.hiddden_channels == [128] * 4 and cfg.model.heads == 2
    assert cfg.model.compile is True and cfg.dataset.batch_size == 10000
    assert cfg.dataset.transforms[0].name == "KNNGraph"
    m = _fill_and_build(cfg)
    assert isinstance(m, GATModule) and m.is_regression
    want = ref.GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).state_dict()
    # compile=True: the model is torch.compile'd as in the reference (gat.py:84), so its keys
    # carry the `_orig_mod.` prefix exactly as the reference's compiled module's do
    assert {k: v.shape for k, v in m.model.state_dict().items()} == \
        {"_orig_mod." + k: v.shape for k, v in want.items()}


def test_parse_args_requires_config(tmp_path):
    from lesion_gnn_amd.utils.config import parse_args

    f = tmp_path / "exp2.py"
    f.write_text(EXPERIMENT)
    with pytest.warns(UserWarning):
        cfg = parse_args(["--config", str(f), "--model.lr", "3"])
    assert cfg.seed == 7
    with pytest.raises(SystemExit):
        parse_args([])
