"""The go-aoi interface GoWorld's engine/entity uses, mirrored over the MI355X engine.

Reference surface (go-aoi v0.2.0, rev 5e9d879, /root/reference/Gopkg.lock:155-159; module not
vendored, names as used by goworld):

    type Coord float32
    type AOI struct { x, y, dist Coord; Data interface{}; callback AOICallback; implData ... }
    func InitAOI(aoi *AOI, dist Coord, data interface{}, callback AOICallback)     # Entity.go:210
    type AOICallback interface { OnEnterAOI(other *AOI); OnLeaveAOI(other *AOI) }  # Entity.go:227-233
    type AOIManager interface { Enter(aoi *AOI, x, y Coord); Leave(aoi *AOI); Moved(aoi *AOI, x, y Coord) }
    func NewXZListAOIManager(aoidist Coord) AOIManager                              # Space.go:105

Differences, all by design of the tick-batched engine (DESIGN.md "Boundary"):
  * Moved() only writes the call into the manager's pinned staging arrays (gwaoi_stage_buffers); the
    batch goes to the GPU in ONE gwaoi_stage_moves_pinned before the next Enter/Leave and at Flush(),
    as the cgo wrapper does. Callbacks of staged moves fire at Flush(), which GoWorld calls once per
    game tick before CollectEntitySyncInfos (GameService.go:185-191). With sync_enter_leave=True
    (default) Enter() and Leave() flush immediately, so their callbacks fire inside the call as in
    the reference (Space.enter runs user hooks right after aoiMgr.Enter, Space.go:211-217).
  * Events are replayed in canonical order (op order, LEAVE before ENTER, other slot ascending);
    inside one Moved the reference's order is Go map iteration order (random).
  * Misuse the reference panics on (Enter twice, Leave/Moved of an AOI not in the manager) raises
    GwaoiError with code GWAOI_ERR_STATE.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, List, Optional, Sequence

from . import _lib
from .engine import Engine

Coord = float


class AOICallback(ABC):
    @abstractmethod
    def OnEnterAOI(self, other: "AOI") -> None: ...

    @abstractmethod
    def OnLeaveAOI(self, other: "AOI") -> None: ...


class AOI:
    __slots__ = ("x", "y", "dist", "Data", "callback", "_slot", "_mgr")

    def __init__(self):
        self.x = 0.0
        self.y = 0.0
        self.dist = 0.0
        self.Data: Any = None
        self.callback: Optional[AOICallback] = None
        self._slot = -1
        self._mgr = None


def InitAOI(aoi: AOI, dist: Coord, data: Any, callback: AOICallback) -> None:
    """go-aoi InitAOI (called at Entity.go:210). `dist` is stored, and — as in the XZ list manager —
    not used: the manager-wide distance applies (TODO.md:19 in the reference)."""
    aoi.dist = dist
    aoi.Data = data
    aoi.callback = callback


class AOIManager(ABC):
    @abstractmethod
    def Enter(self, aoi: AOI, x: Coord, y: Coord) -> None: ...

    @abstractmethod
    def Leave(self, aoi: AOI) -> None: ...

    @abstractmethod
    def Moved(self, aoi: AOI, x: Coord, y: Coord) -> None: ...


class GPUAOIManager(AOIManager):
    """AOIManager backed by libgwaoi on one MI355X. `y` is GoWorld's Z (Space.go:211: aoi.Coord(pos.Z))."""

    def __init__(self, aoidist: Coord, capacity: int = 1 << 16, device: int = 0,
                 bounds: Optional[Sequence[float]] = None, sync_enter_leave: bool = True):
        if not aoidist > 0:
            raise ValueError("aoidist must be > 0 (Space.EnableAOI panics otherwise, Space.go:92-94)")
        self.aoidist = float(aoidist)
        self._eng = Engine(aoidist, capacity=capacity, device=device, bounds=bounds)
        self._by_slot: List[Optional[AOI]] = [None] * capacity
        self._free = list(range(capacity - 1, -1, -1))
        self._released: List[int] = []
        self.sync_enter_leave = sync_enter_leave
        self.last_events = None
        self._ms, self._mx, self._mz = self._eng.stage_buffers()  # pinned, library-owned
        self._nmv = 0  # Moved calls written and not yet pushed

    def _push_moves(self) -> None:
        """One gwaoi_stage_moves_pinned for the Moved calls written since the last push (validated on the
        device; a slot moved twice splits into sub-passes there)."""
        if self._nmv:
            n, self._nmv = self._nmv, 0
            self._eng.stage_moves_pinned(n)

    @property
    def engine(self) -> Engine:
        return self._eng

    def Enter(self, aoi: AOI, x: Coord, y: Coord) -> None:
        if aoi._mgr is not None:
            raise _lib.GwaoiError(_lib.GWAOI_ERR_STATE, "Enter: AOI already in a manager")
        if not self._free:
            raise _lib.GwaoiError(_lib.GWAOI_ERR_NOMEM, "Enter: manager capacity exhausted")
        slot = self._free.pop()
        self._push_moves()  # Moved calls made before this Enter come first
        self._eng.enter(slot, x, y)
        aoi._slot, aoi._mgr = slot, self
        aoi.x, aoi.y = float(x), float(y)
        self._by_slot[slot] = aoi
        if self.sync_enter_leave:
            self.Flush()

    def Leave(self, aoi: AOI) -> None:
        if aoi._mgr is not self:
            raise _lib.GwaoiError(_lib.GWAOI_ERR_STATE, "Leave: AOI not in this manager")
        self._push_moves()
        self._eng.leave(aoi._slot)
        self._released.append(aoi._slot)
        aoi._mgr = None
        if self.sync_enter_leave:
            self.Flush()

    def Moved(self, aoi: AOI, x: Coord, y: Coord) -> None:
        if aoi._mgr is not self:
            raise _lib.GwaoiError(_lib.GWAOI_ERR_STATE, "Moved: AOI not in this manager")
        k = self._nmv
        self._ms[k], self._mx[k], self._mz[k] = aoi._slot, x, y
        self._nmv = k + 1
        if self._nmv == len(self._ms):
            self._push_moves()
        aoi.x, aoi.y = float(x), float(y)

    def Flush(self) -> int:
        """Run the tick and replay its events into the callbacks; returns the number of pair events."""
        self._push_moves()
        ev = self._eng.tick()
        self.last_events = ev
        by = self._by_slot
        for mover, other in ev.tolist():
            a = by[mover]
            o = by[other & _lib.GWAOI_EV_SLOT_MASK]
            if other & _lib.GWAOI_EV_ENTER:
                a.callback.OnEnterAOI(o)  # aoi.callback.OnEnterAOI(neighbor.aoi)
                o.callback.OnEnterAOI(a)  # neighbor.aoi.callback.OnEnterAOI(aoi.aoi)
            else:
                a.callback.OnLeaveAOI(o)
                o.callback.OnLeaveAOI(a)
        for slot in self._released:  # slots are reusable only after their events were replayed
            self._by_slot[slot] = None
            self._free.append(slot)
        self._released.clear()
        return len(ev)

    def close(self):
        self._ms = self._mx = self._mz = None
        self._eng.close()


def NewXZListAOIManager(aoidist: Coord, **kw) -> GPUAOIManager:
    """Drop-in for go-aoi's constructor (Space.go:105): same argument, GPU-backed manager."""
    return GPUAOIManager(aoidist, **kw)
