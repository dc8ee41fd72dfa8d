"""diffusers 0.35.1 ConfigMixin / register_to_config, reduced to what Transformer3DModel and
RectifiedFlowScheduler use: `from_config(dict)` ignores keys the constructor does not take
(e.g. `_class_name`, `project_to_2d_pos`), and `.config` exposes the bound init arguments."""
import functools
import inspect


class FrozenDict(dict):
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as exc:
            raise AttributeError(name) from exc


class ConfigMixin:
    config_name = "config.json"

    @classmethod
    def from_config(cls, config=None, **kwargs):
        merged = dict(config or {})
        merged.update(kwargs)
        accepted = inspect.signature(cls.__init__).parameters
        init_kwargs = {k: v for k, v in merged.items() if k in accepted and k != "self"}
        return cls(**init_kwargs)

    @property
    def config(self):
        return self._internal_dict


def register_to_config(init):
    signature = inspect.signature(init)

    @functools.wraps(init)
    def wrapped(self, *args, **kwargs):
        bound = signature.bind(self, *args, **kwargs)
        bound.apply_defaults()
        recorded = {k: v for k, v in bound.arguments.items() if k != "self"}
        init(self, *args, **kwargs)
        object.__setattr__(self, "_internal_dict", FrozenDict(recorded))

    return wrapped
