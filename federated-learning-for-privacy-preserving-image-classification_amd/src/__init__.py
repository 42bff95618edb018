"""Drop-in mirror of the reference package layout (HIP-backed hot path)."""
