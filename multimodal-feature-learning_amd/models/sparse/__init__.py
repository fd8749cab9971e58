"""Mirror of the reference's ``models/sparse`` transformer (Sparse-DETR), SURVEY §8(f) row 2."""
