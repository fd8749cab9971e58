"""reference models/modules (MSDA, position embedding, helpers)."""
