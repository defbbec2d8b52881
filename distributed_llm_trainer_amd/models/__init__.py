from .config import GPTConfig
from .gpt import GPT, count_parameters

__all__ = ["GPTConfig", "GPT", "count_parameters"]
