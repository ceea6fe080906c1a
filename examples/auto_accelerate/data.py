"""Synthetic datasets of the auto_accelerate example (reference:
atorch/examples/auto_accelerate/data.py): constant-pattern toy regression
rows and random-token language-model samples."""

import torch
from modeling import ModelType, get_vocab_size
from torch.utils.data import Dataset


class ToyDataset(Dataset):
    def __init__(self, size, input_size=16, output_size=8):
        self.size, self.input_size, self.output_size = size, input_size, output_size

    def __len__(self):
        return self.size

    def __getitem__(self, idx):
        return {"input": torch.full((self.input_size,), float(idx % 7) / 7.0),
                "label": torch.ones(self.output_size)}


class RandomLMDataset(Dataset):
    def __init__(self, vocab_size, seq_length, size, seed=0):
        self.vocab_size, self.seq_length, self.size, self.seed = vocab_size, seq_length, size, seed

    def __len__(self):
        return self.size

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        src = torch.randint(1, self.vocab_size, (self.seq_length + 1,), generator=g)
        return {"input_ids": src, "labels": src.clone()}


def get_dataset(model_type, seq_length=16, input_size=16, output_size=8, datasize=200):
    if model_type == ModelType.TOY:
        return ToyDataset(datasize, input_size, output_size)
    return RandomLMDataset(get_vocab_size(model_type), seq_length, datasize)


def get_dataloader_args(model_type, batch_size=8):
    return {"batch_size": batch_size, "drop_last": True, "shuffle": True, "num_workers": 0}
