"""Parameter-efficient fine-tuning: LoRA adapters and QLoRA (NF4 base weights on the HIP kernels)."""
from .lora import LoraConfig, LoraLinear, PeftModel, get_peft_model, prepare_model_for_kbit_training
from .quant import BitsAndBytesConfig, NF4Linear, quantize_model_

__all__ = ["LoraConfig", "LoraLinear", "PeftModel", "get_peft_model", "prepare_model_for_kbit_training",
           "BitsAndBytesConfig", "NF4Linear", "quantize_model_"]
