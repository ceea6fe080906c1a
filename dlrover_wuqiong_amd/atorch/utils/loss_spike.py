"""Loss-spike recording and decoding.

``TokenLossSpike.save_loss(file, loss, iter, losses_str=..., sample_infos_str=...)``
appends one line ``time \\t iter \\t loss \\t per-sample losses \\t sample ids``
when the loss exceeds ``min_loss`` after ``min_iter``;
``decode_loss_spike(out, tokenizer)`` finds, for every recorded spike, the
sample with the largest loss and writes its decoded text (samples are read
by memory-mapping the token file, never loaded whole).  ``fetch`` is the
customisation point mapping a sample id to (dataset name, token ids).

Parity: ATorch ``atorch/utils/loss_spike_utils.py`` (``LossSpikeBase``,
``TokenLossSpike``: save_loss / decode_loss_spike / parse_sample_content /
fetch with ``{scatter_id}-{dsid}-{idx}-{raw_id}-{sample_id}`` ids).
"""

import datetime
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ...common.log import logger


class LossSpikeBase:
    def __init__(self, loss_spike_save_dir: str, sample_data_paths: Sequence[Tuple[str, str]], each_sample_len: int,
                 min_iter: int, min_loss: float, loss_info_splitter: str = "\t", loss_sample_str_splitter: str = ","):
        if not os.path.exists(loss_spike_save_dir):
            raise ValueError("loss_spike_save_dir does not exist")
        self.loss_spike_save_dir = loss_spike_save_dir
        self.sample_data_paths = list(sample_data_paths)
        self.each_sample_len = each_sample_len
        self.min_iter, self.min_loss = min_iter, min_loss
        self.loss_info_splitter = loss_info_splitter
        self.loss_sample_str_splitter = loss_sample_str_splitter

    @staticmethod
    def get_data_file_len(fpath: str, dtype) -> int:
        return os.path.getsize(fpath) // np.dtype(dtype).itemsize


class TokenLossSpike(LossSpikeBase):
    def save_loss(self, file_name: str, cur_loss: float, cur_iter: int, *args, losses_str: str = "",
                  sample_infos_str: str = "", **kwargs) -> bool:
        if not (cur_loss > self.min_loss and cur_iter > self.min_iter):
            return False
        t = datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        line = self.loss_info_splitter.join([t, str(cur_iter), str(cur_loss), losses_str, sample_infos_str])
        with open(os.path.join(self.loss_spike_save_dir, file_name), "a+") as f:
            f.write(line + "\n")
        logger.info(f"loss spike recorded: iter {cur_iter} loss {cur_loss}")
        return True

    def decode_loss_spike(self, result_file_path: str, tokenizer=None, min_iter: Optional[int] = None,
                          min_loss: Optional[float] = None) -> int:
        min_iter = self.min_iter if min_iter is None else min_iter
        min_loss = self.min_loss if min_loss is None else min_loss
        n = 0
        with open(result_file_path, "w") as fw:
            for fname in sorted(os.listdir(self.loss_spike_save_dir)):
                with open(os.path.join(self.loss_spike_save_dir, fname)) as fr:
                    for line in fr:
                        parts = line.rstrip("\n").split(self.loss_info_splitter)
                        if len(parts) < 5:
                            continue
                        it, loss = int(parts[1]), float(parts[2])
                        if it < min_iter or loss < min_loss:
                            continue
                        ds, text, max_loss = self.parse_sample_content(parts[3], parts[4], tokenizer)
                        if ds is None:
                            continue
                        fw.write(f"=========={ds}  {max_loss}================\n{text}\n\n\n\n")
                        n += 1
        return n

    def parse_sample_content(self, losses_str: str, sample_infos_str: str, tokenizer=None):
        losses = [float(x) for x in losses_str.split(self.loss_sample_str_splitter)]
        infos = sample_infos_str.split(self.loss_sample_str_splitter)
        if len(losses) != len(infos):
            logger.warning("batch loss length != batch sample length")
            return None, None, None
        i = int(np.argmax(losses))
        ds, data = self.fetch(infos[i])
        if ds is None:
            return None, None, None
        if tokenizer is not None:
            data = tokenizer.decode(list(map(int, data)))
        return ds, data, losses[i]

    def fetch(self, each_sample_info: str):
        scatter_id, dsid, _idx, _raw, sample_id = each_sample_info.split("-")
        name, base = self.sample_data_paths[int(dsid)]
        path = f"{base}.scatter/{scatter_id}.lazy/text"
        if not os.path.exists(path):
            logger.warning(f"sample data path {path} does not exist")
            return None, None
        n = self.get_data_file_len(path, np.int32) // self.each_sample_len
        mm = np.memmap(path, dtype=np.int32, mode="r", shape=(n, self.each_sample_len))
        return name, np.array(mm[int(sample_id)])


def losses_to_str(losses: List[float], sep: str = ",") -> str:
    return sep.join(f"{x:.6f}" for x in losses)
