"""State-dict shapes of the models BASELINE.json's configurations aggregate.

Only the payload *shapes* matter to the aggregation path (SURVEY.md §8 table
C1-C5), so these are shape lists ``[(key, shape, 'f32'|'i64'), ...]`` in the
models' ``state_dict`` order, not models.  They restate the module structure
of the reference zoo:

* LeNet-5: ``plato/models/lenet5.py:20-47`` (C1).
* CIFAR ResNet-18/34/50/101/152: ``plato/models/resnet.py:14-127,168-189``
  (C2, C3, C4).
* ViT-L/16-shaped and GPT-2-medium-shaped transformers (C5): the reference
  fetches these by name (``models/vit.py``, ``models/huggingface.py``); the
  shapes follow the HuggingFace ViT / GPT-2 module layout at
  hidden 1024, 24 layers, 16 heads, MLP 4096.

``tests/test_workloads.py`` checks the ResNet/LeNet lists against key/shape
fixtures dumped from the reference models (``tests/golden/shapes_*.json``).
"""

from __future__ import annotations

F32 = "f32"
I64 = "i64"


def _bn(prefix: str, c: int):
    return [
        (f"{prefix}.weight", (c,), F32),
        (f"{prefix}.bias", (c,), F32),
        (f"{prefix}.running_mean", (c,), F32),
        (f"{prefix}.running_var", (c,), F32),
        (f"{prefix}.num_batches_tracked", (), I64),
    ]


def lenet5(num_classes: int = 10):
    return [
        ("conv1.weight", (6, 1, 5, 5), F32),
        ("conv1.bias", (6,), F32),
        ("conv2.weight", (16, 6, 5, 5), F32),
        ("conv2.bias", (16,), F32),
        ("conv3.weight", (120, 16, 5, 5), F32),
        ("conv3.bias", (120,), F32),
        ("fc4.weight", (84, 120), F32),
        ("fc4.bias", (84,), F32),
        ("fc5.weight", (num_classes, 84), F32),
        ("fc5.bias", (num_classes,), F32),
    ]


_RESNET_CFG = {
    18: ("basic", (2, 2, 2, 2)),
    34: ("basic", (3, 4, 6, 3)),
    50: ("bottleneck", (3, 4, 6, 3)),
    101: ("bottleneck", (3, 4, 23, 3)),
    152: ("bottleneck", (3, 8, 36, 3)),
}


def resnet(depth: int = 18, num_classes: int = 10):
    """CIFAR-style ResNet (3x3 stem, no max-pool) as in plato/models/resnet.py."""
    kind, blocks = _RESNET_CFG[depth]
    expansion = 1 if kind == "basic" else 4
    spec = [("conv1.weight", (64, 3, 3, 3), F32)] + _bn("bn1", 64)
    in_planes = 64
    for li, (planes, nblocks, stride0) in enumerate(
        zip((64, 128, 256, 512), blocks, (1, 2, 2, 2)), start=1
    ):
        for bi in range(nblocks):
            stride = stride0 if bi == 0 else 1
            p = f"layer{li}.{bi}"
            if kind == "basic":
                spec += [(f"{p}.conv1.weight", (planes, in_planes, 3, 3), F32)] + _bn(f"{p}.bn1", planes)
                spec += [(f"{p}.conv2.weight", (planes, planes, 3, 3), F32)] + _bn(f"{p}.bn2", planes)
            else:
                spec += [(f"{p}.conv1.weight", (planes, in_planes, 1, 1), F32)] + _bn(f"{p}.bn1", planes)
                spec += [(f"{p}.conv2.weight", (planes, planes, 3, 3), F32)] + _bn(f"{p}.bn2", planes)
                spec += [(f"{p}.conv3.weight", (planes * 4, planes, 1, 1), F32)] + _bn(
                    f"{p}.bn3", planes * 4
                )
            out = planes * expansion
            if stride != 1 or in_planes != out:
                spec += [(f"{p}.shortcut.0.weight", (out, in_planes, 1, 1), F32)] + _bn(
                    f"{p}.shortcut.1", out
                )
            in_planes = out
    spec += [("linear.weight", (num_classes, 512 * expansion), F32), ("linear.bias", (num_classes,), F32)]
    return spec


def vit_large(image: int = 224, patch: int = 16, hidden: int = 1024, layers: int = 24,
              mlp: int = 4096, num_labels: int = 10):
    """ViT-L/16-shaped classifier (HuggingFace ViTForImageClassification layout)."""
    n_patches = (image // patch) ** 2
    spec = [
        ("vit.embeddings.cls_token", (1, 1, hidden), F32),
        ("vit.embeddings.position_embeddings", (1, n_patches + 1, hidden), F32),
        ("vit.embeddings.patch_embeddings.projection.weight", (hidden, 3, patch, patch), F32),
        ("vit.embeddings.patch_embeddings.projection.bias", (hidden,), F32),
    ]
    for i in range(layers):
        p = f"vit.encoder.layer.{i}"
        for name in ("query", "key", "value"):
            spec += [
                (f"{p}.attention.attention.{name}.weight", (hidden, hidden), F32),
                (f"{p}.attention.attention.{name}.bias", (hidden,), F32),
            ]
        spec += [
            (f"{p}.attention.output.dense.weight", (hidden, hidden), F32),
            (f"{p}.attention.output.dense.bias", (hidden,), F32),
            (f"{p}.intermediate.dense.weight", (mlp, hidden), F32),
            (f"{p}.intermediate.dense.bias", (mlp,), F32),
            (f"{p}.output.dense.weight", (hidden, mlp), F32),
            (f"{p}.output.dense.bias", (hidden,), F32),
            (f"{p}.layernorm_before.weight", (hidden,), F32),
            (f"{p}.layernorm_before.bias", (hidden,), F32),
            (f"{p}.layernorm_after.weight", (hidden,), F32),
            (f"{p}.layernorm_after.bias", (hidden,), F32),
        ]
    spec += [
        ("vit.layernorm.weight", (hidden,), F32),
        ("vit.layernorm.bias", (hidden,), F32),
        ("classifier.weight", (num_labels, hidden), F32),
        ("classifier.bias", (num_labels,), F32),
    ]
    return spec


def gpt2_medium(vocab: int = 50257, positions: int = 1024, hidden: int = 1024, layers: int = 24):
    """GPT-2-medium-shaped LM (HuggingFace GPT2LMHeadModel layout, tied lm_head listed)."""
    spec = [
        ("transformer.wte.weight", (vocab, hidden), F32),
        ("transformer.wpe.weight", (positions, hidden), F32),
    ]
    for i in range(layers):
        p = f"transformer.h.{i}"
        spec += [
            (f"{p}.ln_1.weight", (hidden,), F32),
            (f"{p}.ln_1.bias", (hidden,), F32),
            (f"{p}.attn.c_attn.weight", (hidden, 3 * hidden), F32),
            (f"{p}.attn.c_attn.bias", (3 * hidden,), F32),
            (f"{p}.attn.c_proj.weight", (hidden, hidden), F32),
            (f"{p}.attn.c_proj.bias", (hidden,), F32),
            (f"{p}.ln_2.weight", (hidden,), F32),
            (f"{p}.ln_2.bias", (hidden,), F32),
            (f"{p}.mlp.c_fc.weight", (hidden, 4 * hidden), F32),
            (f"{p}.mlp.c_fc.bias", (4 * hidden,), F32),
            (f"{p}.mlp.c_proj.weight", (4 * hidden, hidden), F32),
            (f"{p}.mlp.c_proj.bias", (hidden,), F32),
        ]
    spec += [
        ("transformer.ln_f.weight", (hidden,), F32),
        ("transformer.ln_f.bias", (hidden,), F32),
        ("lm_head.weight", (vocab, hidden), F32),
    ]
    return spec


def numel(spec, region: str | None = None) -> int:
    total = 0
    for _, shape, reg in spec:
        if region is None or reg == region:
            n = 1
            for d in shape:
                n *= d
            total += n
    return total


# BASELINE.json configurations -> (model spec, K clients, GPUs)
CONFIGS = {
    "C1": dict(model="lenet5", spec=lambda: lenet5(10), k=10, gpus=0),
    "C2": dict(model="resnet18", spec=lambda: resnet(18, 10), k=128, gpus=1),
    "C3": dict(model="resnet50-200cls", spec=lambda: resnet(50, 200), k=1024, gpus=8),
    "C4": dict(model="resnet18", spec=lambda: resnet(18, 10), k=256, gpus=1),
    "C5": dict(model="vit-large-10cls", spec=lambda: vit_large(), k=32, gpus=8),
    "C5-gpt2": dict(model="gpt2-medium", spec=lambda: gpt2_medium(), k=32, gpus=8),
}
