//go:build !mirsha
// +build !mirsha

// The GPU-batched hash API for builds without the mirsha build tag: the same
// exported declarations as gpuhash.go, no cgo and no libmirsha, so the patched
// reference tree builds and tests exactly as before (.travis.yml:19-20: ginkgo
// -r --race, staticcheck ./...; also CGO_ENABLED=0). NewGPUHasher fails, so a
// node never holds a GPUHasher and ProcessorConfig.GPUHasher stays nil: every
// hash action takes ProcessHashActions (serial.go:180-198) as in the reference.
//
// Go 1.15 compatible (go.mod:3).
package processor

import (
	"github.com/pkg/errors"

	"github.com/hyperledger-labs/mirbft/pkg/statemachine"
)

// errNoMirsha is what every entry point returns in this build. The code is
// MSHA_ERR_NO_DEVICE (2), as libmirsha reports on a host without a GPU.
var errNoMirsha = errors.New("libmirsha error 2: built without the mirsha build tag (go build -tags mirsha)")

// GPUHasher is the libmirsha-backed batch hasher of gpuhash.go; in this build
// no value of it can be created.
type GPUHasher struct{}

// NewGPUHasher always fails in this build (see errNoMirsha).
func NewGPUHasher(deviceMask uint32) (*GPUHasher, error) {
	return nil, errNoMirsha
}

// Close does nothing in this build.
func (g *GPUHasher) Close() {}

// RequestDigests always fails in this build.
func (g *GPUHasher) RequestDigests(reqs []ProposedRequest) ([][]byte, error) {
	return nil, errNoMirsha
}

// ProcessHashActionsGPU always fails in this build; callers that hold no
// GPUHasher use ProcessHashActions.
func ProcessHashActionsGPU(g *GPUHasher, actions *statemachine.ActionList) (*statemachine.EventList, error) {
	return nil, errNoMirsha
}
