"""Planner output types (reference ``pkg/tensorflow/types.go:16-34``)."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import List


class Action(enum.Enum):
    ShouldAddPS = "ShouldAddPS"
    ShouldAddPSService = "ShouldAddPSService"
    ShouldAddWorker = "ShouldAddWorker"
    ShouldAddWorkerService = "ShouldAddWorkerService"
    ShouldDelete = "ShouldDelete"  # declared, never emitted (as in the reference)
    Nothing = "Nothing"


@dataclass
class Event:
    action: Action
    number: int = 0
    # replica indices to create (extension: the reference always creates 0..number-1)
    indices: List[int] = field(default_factory=list)

    def __post_init__(self):
        if self.number and not self.indices:
            self.indices = list(range(self.number))
