"""Model registry (reference: model/model_factory.py:13-64)."""
import os

import numpy as np
import torch

from model.unet_attention import AttentionUNet
from model.unet_dualdense import DualDenseUNet
from model.unet_multitask import MultiTaskUNet
from model.unet_plain import UNetPlain
from model.unet_resnet import Unet as UNetResNet50

SUPPORTED_MODELS = {
    "unet_plain": UNetPlain,
    "unet_resnet50": UNetResNet50,
    "attention_unet": AttentionUNet,
    "dualdense_unet": DualDenseUNet,
    "multitask_unet": MultiTaskUNet,
}


def build_model(model_name: str, num_classes: int, num_seg_classes: int = 1, num_cls_classes: int = 3):
    """model_factory.py:22-38 (ValueError on an unknown name)."""
    if model_name not in SUPPORTED_MODELS:
        raise ValueError(f"Unsupported model: {model_name}. Supported: {sorted(SUPPORTED_MODELS.keys())}")
    if model_name == "multitask_unet":
        return SUPPORTED_MODELS[model_name](num_seg_classes=num_seg_classes, num_cls_classes=num_cls_classes)
    return SUPPORTED_MODELS[model_name](num_classes=num_classes)


def create_model(model_name, num_classes, weights="", num_seg_classes=1, num_cls_classes=3):
    """Alias named by BASELINE.json's north_star (the reference's is train.create_model)."""
    from model.unet_training import weights_init

    model = build_model(model_name, num_classes, num_seg_classes, num_cls_classes)
    weights_init(model)
    if weights:
        load_weights_flexible(model, weights)
    return model


def load_weights_flexible(model, weights_path: str):
    """model_factory.py:41-64: load entries whose key AND shape match, skip the rest."""
    if not weights_path:
        return model
    if not os.path.exists(weights_path):
        raise FileNotFoundError(f"Weights not found: {weights_path}")
    model_dict = model.state_dict()
    pretrained = torch.load(weights_path, map_location="cpu", weights_only=True)
    load_key, no_load_key, temp = [], [], {}
    for k, v in pretrained.items():
        if k in model_dict and np.shape(model_dict[k]) == np.shape(v):
            temp[k] = v
            load_key.append(k)
        else:
            no_load_key.append(k)
    model_dict.update(temp)
    model.load_state_dict(model_dict)
    print(f"Loaded weights: {len(load_key)} keys, Skipped: {len(no_load_key)} keys")
    return model
