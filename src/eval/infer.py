"""Reference-path entry point: ``python src/eval/infer.py --checkpoint ckpt.pt ...``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.eval.infer import main  # noqa: E402

if __name__ == "__main__":
    main()
