"""gallocy_amd — MI355X-native engine for gallocy's DSM hot path (twin / run diff / apply /
batched page coherence). See DESIGN.md and docs/SPEC.md."""
from .gdsm import (CURRENT, GEN_CLUSTERED, GEN_UNIFORM, MAX_RECORD, PAGE_SZ, REPLICA, TWIN,
                   Context, DeviceBuffer, HostRuns, Runs, Tracker, device_count, diff,
                   set_diff_device, version)

__all__ = ["CURRENT", "GEN_CLUSTERED", "GEN_UNIFORM", "MAX_RECORD", "PAGE_SZ", "REPLICA", "TWIN",
           "Context", "DeviceBuffer", "HostRuns", "Runs", "Tracker", "device_count", "diff",
           "set_diff_device", "version"]
