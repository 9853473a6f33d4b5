from .config import (LLAMA31_70B, LLAMA31_8B, MIXTRAL_8X7B, TINY_LLAMA, TINY_MIXTRAL, ModelConfig,
                     get_config, rope_table)

__all__ = ["LLAMA31_70B", "LLAMA31_8B", "MIXTRAL_8X7B", "TINY_LLAMA", "TINY_MIXTRAL", "ModelConfig",
           "get_config", "rope_table"]
