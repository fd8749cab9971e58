"""reference models/deformable (uni- and multimodal deformable transformers)."""
