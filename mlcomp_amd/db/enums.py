"""Enumerations stored as integers in the DB (values identical to the reference,
`mlcomp/db/enums.py:5-74`, so an existing database reads the same)."""
from enum import Enum
import re


def to_snake(name: str) -> str:
    return re.sub(r'(?<!^)(?=[A-Z])', '_', name).lower()


class OrderedEnum(Enum):
    def __ge__(self, other):
        return self.value >= other.value if self.__class__ is other.__class__ else NotImplemented

    def __gt__(self, other):
        return self.value > other.value if self.__class__ is other.__class__ else NotImplemented

    def __le__(self, other):
        return self.value <= other.value if self.__class__ is other.__class__ else NotImplemented

    def __lt__(self, other):
        return self.value < other.value if self.__class__ is other.__class__ else NotImplemented

    @classmethod
    def names(cls):
        return [e.name for e in cls]

    @classmethod
    def names_snake(cls):
        return [to_snake(n) for n in cls.names()]

    @classmethod
    def from_name(cls, name: str) -> int:
        """Value for a CamelCase or snake_case member name."""
        if '_' in name or not name[0].isupper():
            return list(cls)[cls.names_snake().index(name)].value
        return cls[name].value


class DagType(OrderedEnum):
    Standard = 0
    Pipe = 1


class TaskStatus(OrderedEnum):
    NotRan = 0
    Queued = 1
    InProgress = 2
    Failed = 3
    Stopped = 4
    Skipped = 5
    Success = 6


class TaskType(OrderedEnum):
    User = 0
    Train = 1
    Service = 2


class ComponentType(OrderedEnum):
    API = 0
    Supervisor = 1
    Worker = 2
    WorkerSupervisor = 3
    Client = 4


class LogStatus(OrderedEnum):
    Debug = 10
    Info = 20
    Warning = 30
    Error = 40
