"""Data-side configuration surface of the reference (src/lesion_gnn/datasets): the config
dataclasses that an experiment file such as configs/config.py builds (DataConfig, DDRConfig,
AptosConfig, LesionsNodesConfig, ...), with the reference's names and fields, so the file loads
unchanged against this package (utils.config.get_config). The datasets themselves (DDR / APTOS
image folders, the segmentation / timm feature extraction) are out of scope: the
build feeds the hot path synthetic lesion graphs (synth.py). The one data-side kernel in scope,
the per-component feature pooling of the node extractor, is nodes.lesions.extract_features_by_cc.
"""
