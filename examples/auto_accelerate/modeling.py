"""Models of the auto_accelerate example: a toy MLP, GPT-2 and Llama built
from the framework's HIP-kernel layers (random init, no downloads).

Same three model types as the reference example
(atorch/examples/auto_accelerate/modeling.py); the transformer models are the
framework's own (models/gpt2.py, models/llama.py), so fused attention / norms
/ cross-entropy run on the MI355X kernels when a GPU is present.
"""

from enum import Enum, auto

import torch
import torch.nn as nn

from dlrover_wuqiong_amd.models.gpt2 import GPT2, Block, GPT2Config
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer


class ModelType(Enum):
    TOY = auto()
    GPT2 = auto()
    LLAMA = auto()


def get_model_type(name):
    return getattr(ModelType, name.upper(), None)


VOCAB = {ModelType.GPT2: 1024, ModelType.LLAMA: 1024}


def get_vocab_size(model_type):
    return VOCAB[model_type]


class ToyModel(nn.Module):
    def __init__(self, in_features=16, out_features=8, num_linears=3):
        super().__init__()
        self.first_linear = nn.Linear(in_features, out_features)
        self.linears = nn.ModuleList([nn.Linear(out_features, out_features) for _ in range(num_linears - 1)])

    def forward(self, inputs):
        x = self.first_linear(inputs["input"])
        for lin in self.linears:
            x = lin(x)
        return x


class LMWrapper(nn.Module):
    """``model(batch)`` -> loss for the dict batches of data.py."""

    def __init__(self, lm):
        super().__init__()
        self.lm = lm

    def forward(self, input_ids, labels):
        return self.lm(input_ids[:, :-1], labels[:, 1:])


def get_model(model_type, cfg):
    if model_type == ModelType.TOY:
        return ToyModel(cfg["in_features"], cfg["out_features"], cfg["num_linears"])
    if model_type == ModelType.GPT2:
        c = GPT2Config(vocab_size=VOCAB[model_type], n_positions=max(64, cfg["seq_length"]), n_layer=cfg["layer_num"],
                       n_head=cfg["head_num"], n_embd=cfg["hidden_size"])
        return LMWrapper(GPT2(c))
    c = LlamaConfig(vocab_size=VOCAB[model_type], hidden_size=cfg["hidden_size"],
                    intermediate_size=cfg["hidden_size"] * 8 // 3 // 16 * 16 or 16,
                    num_hidden_layers=cfg["layer_num"], num_attention_heads=cfg["head_num"],
                    num_key_value_heads=cfg["head_num"], max_position_embeddings=max(64, cfg["seq_length"]))
    return LMWrapper(Llama(c))


def get_module_type(model_type):
    """The repeated block class (FSDP / activation-checkpoint wrap unit)."""
    return {ModelType.TOY: nn.Linear, ModelType.GPT2: Block, ModelType.LLAMA: LlamaDecoderLayer}[model_type]


def get_model_input_format(model_type):
    return None if model_type == ModelType.TOY else "unpack_dict"


def get_loss_func(model_type):
    if model_type == ModelType.TOY:
        def toy_loss(batch, outputs):
            return nn.functional.mse_loss(outputs, batch["label"])

        return toy_loss

    def lm_loss(batch, outputs):  # the LM wrappers already return the loss
        return outputs

    return lm_loss


def as_tensor_dict(batch):
    return {k: torch.as_tensor(v) for k, v in batch.items()}
