package gwaoi

/*
#include "gwaoi_sync.h"
*/
import "C"

import (
	"unsafe"

	"github.com/xiaonanln/goworld/engine/common"
	"github.com/xiaonanln/goworld/engine/dispatchercluster"
	"github.com/xiaonanln/goworld/engine/netutil"
	"github.com/xiaonanln/goworld/engine/proto"
)

// The two callers either side of the AOI path (include/gwaoi_sync.h, SURVEY 8(f) rows 1-2), on the
// manager's device state. Gate ids are dense indices < nGates <= 256, mapped once by the deployment.

func (g *Manager) EnableSync(nGates int) { chk(C.gwaoi_sync_enable(g.m, C.uint32_t(nGates))) }

// SetEntityID registers the 16-byte EntityID of slot (EntityManager.go:268-270).
func (g *Manager) SetEntityID(slot uint32, id common.EntityID) {
	b := []byte(id) // common.ENTITYID_LENGTH bytes
	s := C.uint32_t(slot)
	chk(C.gwaoi_sync_set_entities(g.m, &s, (*C.uint8_t)(unsafe.Pointer(&b[0])), 1))
}

// SetClient attaches a client (gate index + 16-byte ClientID) to slot; gateIdx = C.GWAOI_SYNC_NO_CLIENT
// detaches it (Entity.SetClient).
func (g *Manager) SetClient(slot uint32, gateIdx uint16, cid common.ClientID) {
	b := []byte(cid)
	s, gi := C.uint32_t(slot), C.uint16_t(gateIdx)
	chk(C.gwaoi_sync_set_clients(g.m, &s, &gi, (*C.uint8_t)(unsafe.Pointer(&b[0])), 1))
}

// SetClientSyncing mirrors Entity.SetClientSyncing (Entity.go:438-440).
func (g *Manager) SetClientSyncing(slot uint32, on bool) {
	s, v := C.uint32_t(slot), C.uint8_t(0)
	if on {
		v = 1
	}
	chk(C.gwaoi_sync_set_syncing(g.m, &s, &v, 1))
}

// HandleSyncPositionYawFromClient replaces GameService.go:398-410 for entities in GPU Spaces: the
// packet payload (32-byte records) goes to the GPU as is; unknown / non-syncing entities are ignored
// exactly as EntityManager.go:482-486 and Entity.go:431-434 ignore them.
func (g *Manager) HandleSyncPositionYawFromClient(payload []byte) {
	if len(payload) == 0 {
		return
	}
	g.pushMoves() // Moved calls made before this packet apply first
	var r C.gwaoi_ingest_result
	chk(C.gwaoi_ingest_positions(g.m, (*C.uint8_t)(unsafe.Pointer(&payload[0])), C.uint64_t(len(payload)),
		C.GWAOI_INGEST_HOST_PAYLOAD, &r))
}

// CollectEntitySyncInfos replaces Entity.go:1221-1267 for entities in GPU Spaces: after Flush, one call
// produces every gate's MT_SYNC_POSITION_YAW_ON_CLIENTS body; the Go side prefixes the msgtype + gateid
// header and sends it.
func (g *Manager) CollectEntitySyncInfos(gateIDs []uint16) {
	var out C.gwaoi_sync_out
	chk(C.gwaoi_collect_sync(g.m, C.GWAOI_COLLECT_HOST, &out))
	off := unsafe.Slice((*uint64)(unsafe.Pointer(out.gate_off)), int(out.n_gates)+1)
	recs := unsafe.Slice((*byte)(unsafe.Pointer(out.records)), int(out.n_records)*48)
	for gi, gateid := range gateIDs {
		if off[gi+1] == off[gi] {
			continue
		}
		pkt := netutil.NewPacket()
		pkt.AppendUint16(proto.MT_SYNC_POSITION_YAW_ON_CLIENTS)
		pkt.AppendUint16(gateid)
		pkt.AppendBytes(recs[off[gi]*48 : off[gi+1]*48])
		dispatchercluster.SelectByGateID(gateid).SendPacket(pkt)
		pkt.Release()
	}
}
