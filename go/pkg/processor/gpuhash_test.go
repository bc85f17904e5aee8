//go:build mirsha
// +build mirsha

// Parity of the GPU-batched hash path against the reference's own CPU path
// (plain `go test`, beside the package's existing suites). Every test skips when
// libmirsha finds no GPU (MSHA_ERR_NO_DEVICE). Built with the mirsha tag only;
// run on a box with a GPU:
//
//	go test -tags mirsha ./pkg/processor/ -run GPU -v
package processor

import (
	"bytes"
	"crypto"
	_ "crypto/sha256"
	"encoding/binary"
	"fmt"
	"strings"
	"testing"

	"google.golang.org/protobuf/proto"

	"github.com/hyperledger-labs/mirbft/pkg/pb/msgs"
	"github.com/hyperledger-labs/mirbft/pkg/pb/state"
	"github.com/hyperledger-labs/mirbft/pkg/statemachine"
)

func newGPU(t *testing.T) *GPUHasher {
	g, err := NewGPUHasher(1)
	if err != nil {
		if strings.Contains(err.Error(), "error 2:") { // MSHA_ERR_NO_DEVICE
			t.Skip(err)
		}
		t.Fatal(err)
	}
	return g
}

func be64(v uint64) []byte {
	b := make([]byte, 8)
	binary.BigEndian.PutUint64(b, v)
	return b
}

// actions: the three producers' encodings (sequence.go:155-172,
// batch_tracker.go:175-188, stateless.go:323-352) plus padding-boundary sizes,
// empty parts and zero-part actions.
func hashActions() *statemachine.ActionList {
	al := &statemachine.ActionList{}
	digest := func(i int) []byte {
		h := crypto.SHA256.New()
		fmt.Fprintf(h, "request-%d", i)
		return h.Sum(nil)
	}
	for k := 0; k <= 20; k++ { // Batch: k request-ack digests
		var data [][]byte
		var acks []*msgs.RequestAck
		for i := 0; i < k; i++ {
			data = append(data, digest(i))
			acks = append(acks, &msgs.RequestAck{ClientId: uint64(i % 4), ReqNo: uint64(i), Digest: digest(i)})
		}
		al.Hash(data, &state.HashOrigin{Type: &state.HashOrigin_Batch_{Batch: &state.HashOrigin_Batch{
			Source: uint64(k % 4), Epoch: 1, SeqNo: uint64(k), RequestAcks: acks}}})
	}
	al.Hash(nil, &state.HashOrigin{Type: &state.HashOrigin_VerifyBatch_{VerifyBatch: &state.HashOrigin_VerifyBatch{
		Source: 1, SeqNo: 9}}}) // empty batch: zero parts
	ec := [][]byte{be64(5), be64(20), bytes.Repeat([]byte{0x11}, 332), be64(4), be64(21), digest(7), be64(4), be64(22), {}}
	al.Hash(ec, &state.HashOrigin{Type: &state.HashOrigin_EpochChange_{EpochChange: &state.HashOrigin_EpochChange{
		Source: 2, Origin: 3}}})
	for _, n := range []int{0, 1, 55, 56, 63, 64, 119, 120, 512, 4097, 65536} {
		al.Hash([][]byte{bytes.Repeat([]byte{byte(n)}, n), {}, []byte("x")}, &state.HashOrigin{})
	}
	return al
}

func TestGPUProcessHashActionsMatchesReference(t *testing.T) {
	g := newGPU(t)
	defer g.Close()
	actions := hashActions()
	want, err := ProcessHashActions(crypto.SHA256, actions)
	if err != nil {
		t.Fatal(err)
	}
	got, err := ProcessHashActionsGPU(g, actions)
	if err != nil {
		t.Fatal(err)
	}
	if got.Len() != want.Len() {
		t.Fatalf("%d results, want %d", got.Len(), want.Len())
	}
	wi, gi, ai := want.Iterator(), got.Iterator(), actions.Iterator()
	for i := 0; i < want.Len(); i++ {
		w, e, a := wi.Next().Type.(*state.Event_HashResult), gi.Next().Type.(*state.Event_HashResult), ai.Next()
		if !bytes.Equal(w.HashResult.Digest, e.HashResult.Digest) {
			t.Errorf("action %d: digest %x, want %x", i, e.HashResult.Digest, w.HashResult.Digest)
		}
		if e.HashResult.Origin != a.Type.(*state.Action_Hash).Hash.Origin {
			t.Errorf("action %d: origin is not the action's pointer", i)
		}
	}
}

// ecHashData restates epochChangeHashData (stateless.go:323-352, unexported
// in package statemachine): [BE64(new_epoch)] ++ [BE64(seq), value] per
// checkpoint ++ [BE64(epoch), BE64(seq), digest] per P and Q entry.
func ecHashData(ec *msgs.EpochChange) [][]byte {
	data := [][]byte{be64(ec.NewEpoch)}
	for _, cp := range ec.Checkpoints {
		data = append(data, be64(cp.SeqNo), cp.Value)
	}
	for _, set := range [][]*msgs.EpochChange_SetEntry{ec.PSet, ec.QSet} {
		for _, e := range set {
			data = append(data, be64(e.Epoch), be64(e.SeqNo), e.Digest)
		}
	}
	return data
}

// An epoch-change storm (epoch_target.go:486-528): every node hashes each of N
// origins' EpochChange once per ack. Acks of the testengine carry the
// originator's message by pointer; acks off the wire carry equal copies; a
// byzantine forwarder may carry an altered one. ProcessHashActionsGPU packs
// each distinct payload once and must still return the reference's digest for
// every action, altered copies included.
func TestGPUEpochChangeStormPackedOnce(t *testing.T) {
	g := newGPU(t)
	defer g.Close()
	const nodes = 16
	al := &statemachine.ActionList{}
	distinct := 0
	for o := 0; o < nodes; o++ {
		ec := &msgs.EpochChange{NewEpoch: 7, Checkpoints: []*msgs.Checkpoint{
			{SeqNo: 500, Value: bytes.Repeat([]byte{byte(o)}, 332)}, {SeqNo: 1000, Value: bytes.Repeat([]byte{byte(o + 1)}, 332)}}}
		for s := 0; s < 300+40*o; s++ {
			ec.PSet = append(ec.PSet, &msgs.EpochChange_SetEntry{Epoch: 6, SeqNo: uint64(s), Digest: bytes.Repeat([]byte{byte(s)}, 32)})
		}
		distinct += partsLen(ecHashData(ec))
		for src := 0; src < nodes; src++ {
			msg := ec // by pointer (the testengine)
			if src%3 == 1 {
				msg = proto.Clone(ec).(*msgs.EpochChange) // an equal copy (off the wire)
			}
			al.Hash(ecHashData(msg), &state.HashOrigin{Type: &state.HashOrigin_EpochChange_{
				EpochChange: &state.HashOrigin_EpochChange{Source: uint64(src), Origin: uint64(o), EpochChange: msg}}})
		}
		bad := proto.Clone(ec).(*msgs.EpochChange) // same origin, same length, one byte differs
		bad.PSet[0].Digest = bytes.Repeat([]byte{0xEE}, 32)
		distinct += partsLen(ecHashData(bad))
		al.Hash(ecHashData(bad), &state.HashOrigin{Type: &state.HashOrigin_EpochChange_{
			EpochChange: &state.HashOrigin_EpochChange{Source: 99, Origin: uint64(o), EpochChange: bad}}})
	}
	want, err := ProcessHashActions(crypto.SHA256, al)
	if err != nil {
		t.Fatal(err)
	}
	got, err := ProcessHashActionsGPU(g, al)
	if err != nil {
		t.Fatal(err)
	}
	wi, gi := want.Iterator(), got.Iterator()
	for i := 0; i < want.Len(); i++ {
		w, e := wi.Next().Type.(*state.Event_HashResult), gi.Next().Type.(*state.Event_HashResult)
		if !bytes.Equal(w.HashResult.Digest, e.HashResult.Digest) {
			t.Fatalf("action %d: digest %x, want %x", i, e.HashResult.Digest, w.HashResult.Digest)
		}
	}
	up, err := g.lastPayloadUpload()
	if err != nil {
		t.Fatal(err)
	}
	// each distinct payload once (plus its 16-byte alignment), not nodes times
	if up < uint64(distinct) || up > uint64(distinct+16*2*nodes) {
		t.Fatalf("uploaded %d payload bytes, distinct payloads hold %d", up, distinct)
	}
}

// One *msgs.EpochChange named by two actions whose Data lists have the same
// length but different bytes (Data built differently from one message, or the
// message changed between the two actions): the pointer alone must not alias
// them (batch_tracker.go:192-195), so each gets the reference's own digest.
func TestGPUEpochChangeSamePointerDifferentData(t *testing.T) {
	g := newGPU(t)
	defer g.Close()
	ec := &msgs.EpochChange{NewEpoch: 3, Checkpoints: []*msgs.Checkpoint{
		{SeqNo: 500, Value: bytes.Repeat([]byte{1}, 332)}}}
	origin := func(src uint64) *state.HashOrigin {
		return &state.HashOrigin{Type: &state.HashOrigin_EpochChange_{
			EpochChange: &state.HashOrigin_EpochChange{Source: src, Origin: 1, EpochChange: ec}}}
	}
	al := &statemachine.ActionList{}
	al.Hash(ecHashData(ec), origin(0))
	other := ecHashData(ec)
	other[0] = be64(4) // same lengths part for part, another new_epoch
	al.Hash(other, origin(1))
	long := ecHashData(ec)
	long[2] = bytes.Repeat([]byte{2}, 332) // a long part from elsewhere, same length
	al.Hash(long, origin(2))
	al.Hash(ecHashData(ec), origin(3)) // the same Data again: aliased
	want, err := ProcessHashActions(crypto.SHA256, al)
	if err != nil {
		t.Fatal(err)
	}
	got, err := ProcessHashActionsGPU(g, al)
	if err != nil {
		t.Fatal(err)
	}
	wi, gi := want.Iterator(), got.Iterator()
	var digests [][]byte
	for i := 0; i < want.Len(); i++ {
		w, e := wi.Next().Type.(*state.Event_HashResult), gi.Next().Type.(*state.Event_HashResult)
		if !bytes.Equal(w.HashResult.Digest, e.HashResult.Digest) {
			t.Fatalf("action %d: digest %x, want %x", i, e.HashResult.Digest, w.HashResult.Digest)
		}
		digests = append(digests, e.HashResult.Digest)
	}
	if bytes.Equal(digests[0], digests[1]) || bytes.Equal(digests[0], digests[2]) || !bytes.Equal(digests[0], digests[3]) {
		t.Fatalf("aliasing by pointer alone: %x", digests)
	}
	reqs := []*state.ActionHashRequest{}
	for it, a := al.Iterator(), (*state.Action)(nil); ; {
		if a = it.Next(); a == nil {
			break
		}
		reqs = append(reqs, a.Type.(*state.Action_Hash).Hash)
	}
	if alias, _ := epochChangeAliases(reqs); alias[1] != -1 || alias[2] != -1 || alias[3] != 0 {
		t.Fatalf("alias = %v, want [-1 -1 -1 0]", alias)
	}
}

func TestGPUProcessHashActionsErrors(t *testing.T) {
	g := newGPU(t)
	defer g.Close()
	al := (&statemachine.ActionList{}).Hash([][]byte{[]byte("x")}, nil)
	al.PushBack(&state.Action{Type: &state.Action_AllocatedRequest{AllocatedRequest: &state.ActionRequestSlot{}}})
	_, want := ProcessHashActions(crypto.SHA256, al)
	_, got := ProcessHashActionsGPU(g, al)
	if want == nil || got == nil || got.Error() != want.Error() {
		t.Fatalf("error %v, want %v", got, want)
	}
	empty, err := ProcessHashActionsGPU(g, &statemachine.ActionList{})
	if err != nil || empty.Len() != 0 {
		t.Fatalf("empty list: %v %v", empty, err)
	}
}

// memStore: a map-backed RequestStore (the testengine's ReqStore shape).
type memStore struct {
	requests    map[string][]byte
	allocations map[[2]uint64][]byte
}

func newMemStore() *memStore {
	return &memStore{requests: map[string][]byte{}, allocations: map[[2]uint64][]byte{}}
}
func (m *memStore) GetAllocation(c, r uint64) ([]byte, error) { return m.allocations[[2]uint64{c, r}], nil }
func (m *memStore) PutAllocation(c, r uint64, d []byte) error {
	m.allocations[[2]uint64{c, r}] = d
	return nil
}
func (m *memStore) GetRequest(a *msgs.RequestAck) ([]byte, error) {
	return m.requests[fmt.Sprintf("%d.%d.%x", a.ClientId, a.ReqNo, a.Digest)], nil
}
func (m *memStore) PutRequest(a *msgs.RequestAck, data []byte) error {
	m.requests[fmt.Sprintf("%d.%d.%x", a.ClientId, a.ReqNo, a.Digest)] = data
	return nil
}
func (m *memStore) Sync() error { return nil }

func TestGPUProposeBatchMatchesPropose(t *testing.T) {
	g := newGPU(t)
	defer g.Close()
	var reqs []ProposedRequest
	for r := uint64(0); r < 300; r++ { // testengine payloads: LE64(client) "-" LE64(reqNo) (recorder.go:258-270)
		b := make([]byte, 17)
		binary.LittleEndian.PutUint64(b, 3)
		b[8] = '-'
		binary.LittleEndian.PutUint64(b[9:], r)
		reqs = append(reqs, ProposedRequest{ReqNo: r, Data: b})
	}
	reqs = append(reqs, ProposedRequest{ReqNo: 5, Data: reqs[5].Data}) // a duplicate: no new events
	mk := func() (*Client, *memStore) {
		s := newMemStore()
		c := (&Clients{Hasher: crypto.SHA256, RequestStore: s}).Client(3)
		for r := uint64(0); r < 300; r += 7 { // some allocated before the proposals
			if _, err := c.allocate(r); err != nil {
				t.Fatal(err)
			}
		}
		return c, s
	}
	cpu, cpuStore := mk()
	want := &statemachine.EventList{}
	for _, r := range reqs {
		el, err := cpu.Propose(r.ReqNo, r.Data)
		if err != nil {
			t.Fatal(err)
		}
		want.PushBackList(el)
	}
	gpu, gpuStore := mk()
	got, err := gpu.ProposeBatch(g, reqs)
	if err != nil {
		t.Fatal(err)
	}
	if got.Len() != want.Len() || got.Len() == 0 {
		t.Fatalf("%d events, want %d", got.Len(), want.Len())
	}
	wi, gi := want.Iterator(), got.Iterator()
	for i := 0; i < want.Len(); i++ {
		w := wi.Next().Type.(*state.Event_RequestPersisted).RequestPersisted.RequestAck
		e := gi.Next().Type.(*state.Event_RequestPersisted).RequestPersisted.RequestAck
		if w.ClientId != e.ClientId || w.ReqNo != e.ReqNo || !bytes.Equal(w.Digest, e.Digest) {
			t.Errorf("event %d: %v, want %v", i, e, w)
		}
	}
	if fmt.Sprint(len(cpuStore.requests), len(cpuStore.allocations)) != fmt.Sprint(len(gpuStore.requests), len(gpuStore.allocations)) {
		t.Fatalf("stores differ")
	}
	for k, v := range cpuStore.allocations {
		if !bytes.Equal(gpuStore.allocations[k], v) {
			t.Errorf("allocation %v: %x, want %x", k, gpuStore.allocations[k], v)
		}
	}
	if n, _ := cpu.NextReqNo(); true {
		if m, _ := gpu.NextReqNo(); m != n {
			t.Errorf("nextReqNo %d, want %d", m, n)
		}
	}
}
