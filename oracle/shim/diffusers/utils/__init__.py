"""diffusers.utils subset: logging, deprecate, is_torch_version, BaseOutput."""
import dataclasses
import logging as _logging
from collections import OrderedDict


class _LoggingShim:
    @staticmethod
    def get_logger(name):
        return _logging.getLogger(name)


logging = _LoggingShim()


def deprecate(*args, **kwargs):
    return None


def is_torch_version(operation, version):
    return True


class BaseOutput(OrderedDict):
    """Dataclass outputs that also index like a tuple / dict (diffusers BaseOutput)."""

    def __post_init__(self):
        for field in dataclasses.fields(self):
            value = getattr(self, field.name)
            if value is not None:
                self[field.name] = value

    def __getitem__(self, key):
        if isinstance(key, int):
            return list(self.values())[key]
        return super().__getitem__(key)

    def to_tuple(self):
        return tuple(self.values())
