"""Callbacks deferred until after pipeline partitioning (reference: trainer/post_partition_hooks.py:5-35)."""

from __future__ import annotations

from typing import Any, Callable, List, Tuple


class PostPartitionHooks:
    def __init__(self):
        self.hooks: List[Tuple[Callable, tuple, dict]] = []

    def register_post_partition_hook(self, func: Callable, func_args: tuple = (), func_kwargs: dict = None) -> None:
        self.hooks.append((func, tuple(func_args), dict(func_kwargs or {})))

    def execute_all_hooks(self, model: Any = None) -> None:
        for func, args, kwargs in self.hooks:
            if model is not None:
                func(*args, model, **kwargs)
            else:
                func(*args, **kwargs)
        self.hooks.clear()
