"""Drop-in replacement of the reference's ``utils`` package (train/eval loops, helpers, synthetic data)."""
