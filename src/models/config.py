"""Reference-path shim: ``models.config.GPTConfig`` (importable with ``src`` on sys.path,
as the reference's scripts expect -- ``src/models/config.py``)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.models.config import GPTConfig  # noqa: E402,F401
