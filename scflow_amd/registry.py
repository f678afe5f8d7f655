"""A ``MODELS`` registry compatible with the one SCFlow builds its decoder from.

Reference: ``registry.py:16`` (``MODELS = Registry('model', parent=MMENGINE_MODELS,
locations=['models'])``) and ``BaseRefiner.__init__`` → ``MODELS.build(decoder)``
(``models/refiner/base_refiner.py:41-42``).  Configs pass ``type`` as a class object
(``configs/refine_models/scflow_ycbv_real.py:208``) or a string (legacy ``raft.py:41``).

mmengine is not installed in this environment (nor guaranteed on the GPU box), so this is a
small self-contained registry with the same ``register_module()`` / ``build(cfg)`` / ``get``
surface.  When mmengine *is* importable, ``register_into_mmengine()`` also registers every
class into a given mmengine registry (e.g. the reference's own ``registry.MODELS``), which is
how a reference checkout adopts these modules without code changes.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional


class Registry:
    def __init__(self, name: str, locations=()):
        self.name = name
        self._modules: Dict[str, type] = {}
        # like mmengine's ``locations``: modules imported on the first lookup miss
        self._locations = list(locations)
        self._imported = False

    def _import_locations(self) -> None:
        if not self._imported:
            import importlib
            self._imported = True
            for loc in self._locations:
                importlib.import_module(loc)

    def __contains__(self, key: str) -> bool:
        return key in self._modules

    def __repr__(self) -> str:
        return f"Registry({self.name}, {sorted(self._modules)})"

    def get(self, key: str) -> Optional[type]:
        if key not in self._modules:
            self._import_locations()
        return self._modules.get(key)

    def register_module(self, name: Optional[str] = None, force: bool = False,
                        module: Optional[type] = None) -> Callable:
        def _register(cls):
            key = name or cls.__name__
            if key in self._modules and not force and self._modules[key] is not cls:
                raise KeyError(f"{key} is already registered in {self.name}")
            self._modules[key] = cls
            return cls
        if module is not None:
            return _register(module)
        return _register

    def build(self, cfg: Dict[str, Any], **default_args) -> Any:
        if not isinstance(cfg, dict) or "type" not in cfg:
            raise TypeError(f"cfg must be a dict with a 'type' key, got {cfg!r}")
        args = dict(cfg)
        typ = args.pop("type")
        if isinstance(typ, str):
            cls = self.get(typ)
            if cls is None:
                raise KeyError(f"{typ} is not registered in {self.name}")
        elif isinstance(typ, type):
            cls = typ
        else:
            raise TypeError(f"type must be a str or a class, got {typ!r}")
        for k, v in default_args.items():
            args.setdefault(k, v)
        return cls(**args)

    def register_into_mmengine(self, target) -> None:
        """Register every class of this registry into an mmengine ``Registry`` ``target``."""
        for key, cls in self._modules.items():
            target.register_module(name=key, module=cls, force=True)


MODELS = Registry("model", locations=["scflow_amd.modules", "scflow_amd.decoder", "scflow_amd.encoder",
                                       "scflow_amd.refiner"])
