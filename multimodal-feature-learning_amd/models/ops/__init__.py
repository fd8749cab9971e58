"""reference models/ops: Python side of the (dormant) MSDA extension."""
