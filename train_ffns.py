"""Reference-compatible entry point: ``python train_ffns.py -s 16 -bs 8 -n 1024 -l 1 -d 8192 -m M``.

Thin wrapper over ``dllm.train_ffns`` (package ``distributed-llm-code-samples_amd/``).  Importing this
module also exposes the reference's module-level API (``init_tlayer_ffn``, ``mock_data``,
``train_1gpu`` / ``train_ddp`` / ``train_fsdp`` / ``train_tp``, ``tlayers_ffn_fwd`` …) from
``dllm.api``, so ``from train_ffns import train_ddp`` keeps working."""
import sys

import dllm  # noqa: F401  (registers the package)
from dllm.api import *  # noqa: F401,F403  (reference-compatible functions)
from dllm.train_ffns import main

if __name__ == "__main__":
    sys.exit(main())
