"""Reference-path entry point: ``python src/training/ddp_trainer.py ...`` or
``torchrun --standalone --nproc_per_node N src/training/ddp_trainer.py ...``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.training.ddp_trainer import *  # noqa: E402,F401,F403
from distributed_llm_trainer_amd.training.ddp_trainer import main  # noqa: E402

if __name__ == "__main__":
    main()
