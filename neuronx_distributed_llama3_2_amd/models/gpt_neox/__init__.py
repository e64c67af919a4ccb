from .modeling_gpt_neox import GPTNeoXForCausalLM, GPTNeoXModel, gpt_neox_config, hf_to_nxd  # noqa: F401
