"""Job status vocabulary and the three mappings the reference components apply.

Internal (brain/ES) statuses, state diagram .gitbook/assets/foremastrequeststatediagram.png:
initial -> preprocess_inprogress -> {completed_health | completed_unhealth |
completed_unknown}; a cycle that ends before endTime leaves the job
``preprocess_completed`` ("reprogress") to be reserved again; ``abort`` is set
by the client; ``preprocess_failed`` for unusable requests.
"""
from __future__ import annotations

from . import crd

INITIAL = "initial"
PREPROCESS_INPROGRESS = "preprocess_inprogress"
POSTPROCESS_INPROGRESS = "postprocess_inprogress"
PREPROCESS_COMPLETED = "preprocess_completed"
PREPROCESS_FAILED = "preprocess_failed"
COMPLETED_HEALTH = "completed_health"
COMPLETED_UNHEALTH = "completed_unhealth"
COMPLETED_UNKNOWN = "completed_unknown"
ABORT = "abort"

TERMINAL = {COMPLETED_HEALTH, COMPLETED_UNHEALTH, COMPLETED_UNKNOWN, PREPROCESS_FAILED, ABORT}
IN_PROGRESS = {PREPROCESS_INPROGRESS, POSTPROCESS_INPROGRESS}
CLAIMABLE = {INITIAL, PREPROCESS_COMPLETED}


def to_external(status: str) -> str:
    """foremast-service/pkg/converter/converter.go:10-29."""
    if status == INITIAL:
        return "new"
    if status in (PREPROCESS_INPROGRESS, POSTPROCESS_INPROGRESS, PREPROCESS_COMPLETED):
        return "inprogress"
    if status == COMPLETED_HEALTH:
        return "success"
    if status == COMPLETED_UNHEALTH:
        return "anomaly"
    if status in (COMPLETED_UNKNOWN, PREPROCESS_FAILED, ABORT):
        return "abort"
    return "unknown"


def to_monitor_phase(status: str) -> str:
    """Barrelman's GetStatus mapping (analystclient.go:226-245); unknown values pass through."""
    if status in ("created", "initial", "new", "inprogress", "unknown"):
        return crd.PHASE_RUNNING
    if status in ("completed_health", "success"):
        return crd.PHASE_HEALTHY
    if status in ("completed_unhealth", "anomaly"):
        return crd.PHASE_UNHEALTHY
    if status == "abort":
        return crd.PHASE_ABORT
    if status == "completed_unknown":
        return crd.PHASE_WARNING
    return status


def to_trigger_phase(status: str) -> str:
    """foremast-trigger's copy of the client (foremast-trigger/pkg/foremasttrigger/analystclient.go:214-229);
    identical vocabulary to barrelman's."""
    return to_monitor_phase(status)
