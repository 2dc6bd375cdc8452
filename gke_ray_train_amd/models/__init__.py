"""Model families: Llama-2/3/3.1 (7B/8B/13B/70B + tiny test configs) and the reference BasicLLM."""
from .basic_llm import BASIC_CONFIGS, BasicLLM, BasicLLMConfig, PositionalEncoding, build_basic_llm
from .llama import CONFIGS, LlamaConfig, LlamaForCausalLM, build_llama, get_config

__all__ = ["BASIC_CONFIGS", "BasicLLM", "BasicLLMConfig", "PositionalEncoding", "build_basic_llm",
           "CONFIGS", "LlamaConfig", "LlamaForCausalLM", "build_llama", "get_config"]
