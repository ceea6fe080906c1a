"""Allow-listed unpickling of checkpoint payloads (no arbitrary code)."""

import argparse
import io
import os
import pickle
from collections import OrderedDict

import numpy as np
import pytest
import torch

from dlrover_wuqiong_amd.common.serialize import restricted_loads, safe_torch_load


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_restricted_loads_refuses_code():
    with pytest.raises(pickle.UnpicklingError):
        restricted_loads(pickle.dumps(_Evil()))
    with pytest.raises(pickle.UnpicklingError):
        restricted_loads(pickle.dumps(eval))


def test_restricted_loads_accepts_checkpoint_objects():
    obj = {"od": OrderedDict(a=1), "ns": argparse.Namespace(lr=1.0), "np": np.arange(3), "dt": torch.float32,
           "rng": np.random.get_state(), "s": {1, 2}, "b": b"x"}
    out = restricted_loads(pickle.dumps(obj))
    assert out["od"] == obj["od"] and out["ns"].lr == 1.0 and out["dt"] is torch.float32
    assert np.array_equal(out["np"], obj["np"])


def test_safe_torch_load_falls_back_to_allow_list(tmp_path):
    p = tmp_path / "x.pt"
    torch.save({"args": argparse.Namespace(tp=8), "w": torch.ones(2)}, p)
    out = safe_torch_load(str(p))
    assert out["args"].tp == 8 and torch.equal(out["w"], torch.ones(2))
    bad = io.BytesIO()
    torch.save({"x": _Evil()}, bad)
    bad.seek(0)
    with pytest.raises(Exception):
        safe_torch_load(bad)


@pytest.mark.parametrize("module,name", [("types", "CodeType"), ("types", "FunctionType"), ("typing", "cast"),
                                         ("functools", "partial"), ("builtins", "getattr"), ("builtins", "type"),
                                         ("builtins", "object"), ("pathlib", "Path"), ("operator", "attrgetter"),
                                         ("torch", "load"), ("numpy", "load"), ("torch.hub", "load")])
def test_restricted_loads_refuses_callable_builders(module, name):
    # GLOBAL <module> <name> ; EMPTY_TUPLE ; REDUCE ; STOP -- the shape of a
    # CodeType/FunctionType chain that would execute attacker bytecode
    payload = b"c" + module.encode() + b"\n" + name.encode() + b"\n)R."
    with pytest.raises(pickle.UnpicklingError):
        restricted_loads(payload)


def test_restricted_loads_dcp_metadata():
    from torch.distributed.checkpoint.metadata import (ChunkStorageMetadata, Metadata, MetadataIndex,
                                                       TensorProperties, TensorStorageMetadata)

    md = Metadata(state_dict_metadata={"w": TensorStorageMetadata(
        properties=TensorProperties(dtype=torch.bfloat16), size=torch.Size([4, 4]),
        chunks=[ChunkStorageMetadata(offsets=torch.Size([0, 0]), sizes=torch.Size([4, 4]))])},
        storage_data={MetadataIndex("w", torch.Size([0, 0]), 0): "x"})
    out = restricted_loads(pickle.dumps(md))
    assert out.state_dict_metadata["w"].size == torch.Size([4, 4])
    assert out.state_dict_metadata["w"].properties.dtype is torch.bfloat16
