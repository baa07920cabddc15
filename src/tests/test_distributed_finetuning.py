"""The reference keeps a second copy of its suite under src/tests/ (SURVEY §0.3);
mxllm keeps a single source of truth in tests/ and re-exports it here."""
from tests.test_distributed_finetuning import TestDistributedFinetuning  # noqa: F401

if __name__ == "__main__":
    import unittest

    unittest.main()
