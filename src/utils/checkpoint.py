"""Reference-path shim for the checkpoint utilities (advertised at README.md:49-52 of
the reference but absent there)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.utils.checkpoint import *  # noqa: E402,F401,F403
