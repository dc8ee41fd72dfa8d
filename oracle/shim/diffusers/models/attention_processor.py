# import-only names referenced by ltx_video/models/transformers/attention.py:9-15
class LoRAAttnAddedKVProcessor:
    pass


class LoRAAttnProcessor:
    pass


class LoRAAttnProcessor2_0:
    pass


class LoRAXFormersAttnProcessor:
    pass


class SpatialNorm:
    pass
