"""Drop-in replacement of the reference's ``model`` package (model_factory, U-Net variants, losses)."""
