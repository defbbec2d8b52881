from .dummy import create_dummy_dataloader
from .openwebtext import create_openwebtext_dataloader
from .tinystories import create_tinystories_dataloader

__all__ = ["create_dummy_dataloader", "create_tinystories_dataloader", "create_openwebtext_dataloader"]
