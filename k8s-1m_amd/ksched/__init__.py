"""ksched — MI355X-native core of dist-scheduler's per-shard Filter/Score/select/commit path.

Python mirror of the host interface; all compute runs in libksched.so (HIP, gfx950).
"""
from . import _abi, objects, synth  # noqa: F401
from .framework import (  # noqa: F401
    FILTER_PLUGINS,
    NODE_PLUGIN_SCORES_STATE_KEY,
    Code,
    CycleState,
    Diagnosis,
    FitError,
    FrameworkError,
    NodePluginScores,
    NodePluginScoresState,
    ScheduleResult,
    Scheduler,
)
from .objects import (  # noqa: F401
    Container,
    Node,
    NodeSelectorRequirement,
    NodeSelectorTerm,
    Pod,
    PreferredSchedulingTerm,
    Taint,
    Toleration,
)
