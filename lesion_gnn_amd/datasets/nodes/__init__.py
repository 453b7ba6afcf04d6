"""Node-extractor configs (reference src/lesion_gnn/datasets/nodes) and the per-component
feature pooling kernel (lesions.extract_features_by_cc)."""
