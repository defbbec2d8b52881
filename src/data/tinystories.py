"""Reference-path shim for ``data.tinystories``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.data.tinystories import *  # noqa: E402,F401,F403
