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
    assert {k: v.shape for k, v in m.model.state_dict().items()} == \
        {k: v.shape for k, v in want.items()}


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
