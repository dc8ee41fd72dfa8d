class LoRACompatibleLinear:  # import-only: never instantiated on the LTX path
    pass
