//go:build !mirsha
// +build !mirsha

// Builds without the mirsha tag: the GPU API is declared but reports that
// libmirsha is not built in, and the callers' CPU path is untouched.
package processor

import (
	"strings"
	"testing"

	"github.com/hyperledger-labs/mirbft/pkg/statemachine"
)

func TestGPUHasherStubReportsNoLibrary(t *testing.T) {
	g, err := NewGPUHasher(1)
	if g != nil || err == nil || !strings.Contains(err.Error(), "-tags mirsha") {
		t.Fatalf("NewGPUHasher = %v, %v; want nil and the build-tag error", g, err)
	}
	al := (&statemachine.ActionList{}).Hash([][]byte{[]byte("x")}, nil)
	if _, err := ProcessHashActionsGPU(nil, al); err == nil {
		t.Fatal("ProcessHashActionsGPU succeeded without libmirsha")
	}
	if _, err := (&Client{}).ProposeBatch(nil, []ProposedRequest{{ReqNo: 1, Data: []byte("x")}}); err == nil {
		t.Fatal("ProposeBatch succeeded without libmirsha")
	}
}
