package gwaoi

import (
	"math/rand"
	"testing"

	"github.com/xiaonanln/go-aoi"
)

// ent is the AOI part of engine/entity's Entity (Entity.go:210, 227-246).
type ent struct {
	aoi  aoi.AOI
	x, z float32
	in   map[*ent]bool
}

func (e *ent) OnEnterAOI(o *aoi.AOI) { e.in[o.Data.(*ent)] = true }
func (e *ent) OnLeaveAOI(o *aoi.AOI) { delete(e.in, o.Data.(*ent)) }

// the reference predicate (go-aoi XZ list manager): o inside the box of the one that acted last,
// bounds float32(c +- D), inclusive. After every Flush each entity's set must equal it.
func inbox(m, o *ent, d float32) bool {
	return o.x >= m.x-d && o.x <= m.x+d && o.z >= m.z-d && o.z <= m.z+d
}

// TestManagerAgainstBruteForce is tests/abi_smoke.c in Go: MySpace's 10 monsters at the origin
// (examples/test_game/MySpace.go:27-34), a lattice crowd with exact-D offsets, then ticks of batched
// moves with one slot moved twice, all moving by small steps so the last actor's box decides.
func TestManagerAgainstBruteForce(t *testing.T) {
	const d = 100
	g := NewXZListAOIManager(d, 96, 0)
	defer g.Close()
	var ents []*ent
	add := func(x, z float32) {
		e := &ent{x: x, z: z, in: map[*ent]bool{}}
		aoi.InitAOI(&e.aoi, d, e, e)
		ents = append(ents, e)
		g.Enter(&e.aoi, aoi.Coord(x), aoi.Coord(z))
	}
	for i := 0; i < 10; i++ {
		add(0, 0)
	}
	for s := 10; s < 60; s++ {
		add(float32((s*37)%9)*50-200, float32((s*11)%7)*50-150)
	}
	check := func(what string) {
		for _, e := range ents {
			for _, o := range ents {
				if e == o {
					continue
				}
				want := inbox(e, o, d) && inbox(o, e, d) // symmetric for these inputs (no rounding ties)
				if e.in[o] != want {
					t.Fatalf("%s: pair state %v, want %v", what, e.in[o], want)
				}
			}
		}
	}
	check("enter")
	r := rand.New(rand.NewSource(12345))
	for tick := 0; tick < 6; tick++ {
		for _, e := range ents {
			e.x += float32(r.Intn(41) - 20)
			e.z += float32(r.Intn(41) - 20)
			g.Moved(&e.aoi, aoi.Coord(e.x), aoi.Coord(e.z))
		}
		e := ents[7]
		e.x++
		g.Moved(&e.aoi, aoi.Coord(e.x), aoi.Coord(e.z)) // the same slot twice in one tick
		g.Flush()
		check("tick")
	}
	g.Leave(&ents[3].aoi)
	for _, e := range ents {
		if e.in[ents[3]] {
			t.Fatalf("leave: still interested in the leaver")
		}
	}
}
