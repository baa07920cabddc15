"""Reference test-suite contract (reference tests/test_distributed_finetuning.py):
the same three tests — custom dataset, process_batch, gpu_tensor_operation —
against ``src.distributed_finetuning`` / ``src.utils``.

Fixture change: the reference calls ``setup(0, 2)`` from ONE
process, so rendezvous waits forever for rank 1.  Here the class fixture
starts a real peer process that joins as rank 1 (gloo on CPU), parks until the
tests finish, then both sides tear the group down.
"""
import multiprocessing as mp
import os
import socket
import unittest

import torch

from src.distributed_finetuning import CustomDataset, cleanup, setup
from src.utils import gpu_tensor_operation, process_batch


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _peer(port, release):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    from src.distributed_finetuning import cleanup as c, setup as s

    s(1, 2)
    release.wait(120)
    c()


class TestDistributedFinetuning(unittest.TestCase):
    @classmethod
    def setUpClass(cls):
        cls.world_size, cls.rank = 2, 0
        port = _free_port()
        cls._saved = {k: os.environ.get(k) for k in ("MASTER_ADDR", "MASTER_PORT", "MXLLM_FORCE_CPU")}
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
        ctx = mp.get_context("spawn")
        cls._release = ctx.Event()
        cls._proc = ctx.Process(target=_peer, args=(port, cls._release), daemon=True)
        cls._proc.start()
        setup(cls.rank, cls.world_size)

    @classmethod
    def tearDownClass(cls):
        cls._release.set()
        cleanup()
        cls._proc.join(60)
        for k, v in cls._saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    def test_custom_dataset(self):
        ds = CustomDataset(["alpha", "beta", "gamma", "delta"], [1, 0, 1, 1])
        self.assertEqual(len(ds), 4)
        item = ds[2]
        self.assertEqual(item["text"], "gamma")
        self.assertEqual(item["label"], 1)

    def test_process_batch(self):
        calls = []

        def fake_llm(prompt):
            calls.append(prompt)
            return "a canned reply"

        loss = process_batch(torch.nn.Linear(1, 1), ["first prompt", "second prompt"], [1, 0], fake_llm)
        self.assertIsInstance(loss, torch.Tensor)
        self.assertEqual(loss.shape, torch.Size([]))
        self.assertEqual(len(calls), 2)

    def test_gpu_tensor_operation(self):
        dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        result = gpu_tensor_operation("test", dev)
        self.assertIsInstance(result, float)
        self.assertAlmostEqual(result, sum(map(ord, "test")) / 4, places=4)


if __name__ == "__main__":
    unittest.main()
