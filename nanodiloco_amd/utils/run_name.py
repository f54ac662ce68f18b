"""Run naming (REF/nanodiloco/training_utils/utils.py:18-39).

Format: ``[debug_]{experiment_type}[_n{nodes}][_{location}]_{MMDD_HHMM}_{uuid8}``.
"""
import uuid
from datetime import datetime
from typing import Any, Dict, Optional


def create_run_name(experiment_type: str, node_config: Dict[str, Any], is_debug: bool = False,
                    now: Optional[datetime] = None) -> str:
    stamp = (now or datetime.now()).strftime("%m%d_%H%M")
    parts = ["debug"] if is_debug else []
    parts.append(experiment_type)
    if node_config.get("nodes"):
        parts.append(f"n{node_config['nodes']}")
    if node_config.get("location"):
        parts.append(str(node_config["location"]))
    parts.append(stamp)
    return "_".join(parts) + "_" + uuid.uuid4().hex[:8]
