//go:build linux && sqobfs

// Package sqobfs binds the MI355X obfuscation library (include/sqobfs.h,
// libsqobfs.so) for sing-quic's Salamander and XPlus decorators
// (hysteria2/salamander.go, hysteria/xplus.go in the reference).
//
// cgo pointer rules: nothing below passes a Go pointer that holds other Go
// pointers, and C never keeps a Go pointer after a call returns.  Byte
// slices passed to C (payloads, the PSK, read buffers) contain no pointers
// and are only used for the duration of the call; batch descriptors and
// datagram slots are C memory.
//
// Lifetimes: a Context is reference counted.  Open returns one with a single
// reference (the caller's); every Keyring and Slots made from it holds
// another, so the C context is closed only after the last of them is closed
// or freed, whatever the order the caller (or a finalizer) uses.  Shared
// hands out one context per GPU to every Conn of the process (Hysteria's
// port hopping re-dials every 30 s, hysteria/hop.go:114; a connection costs
// no new context and no device-wide synchronisation).
//
// Not compiled in the repository's own image (it has no Go toolchain): the C
// call sequences of this package are replayed by tests/cpp/test_cgo_sequence.c
// (Slots) and tests/cpp/test_pconn.c (Conn's engine, sqobfs_pconn_*).
package sqobfs

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/sqobfs/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/sqobfs/lib -lsqobfs -Wl,-rpath,${SRCDIR}/../../third_party/sqobfs/lib
#include <stdlib.h>
#include <string.h>
#include "sqobfs.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"sync"
	"unsafe"
)

// Kind of obfuscation (include/sqobfs.h enum sqobfs_kind).
type Kind int

const (
	Salamander Kind = C.SQOBFS_SALAMANDER // hysteria2/salamander.go
	XPlus      Kind = C.SQOBFS_XPLUS      // hysteria/xplus.go
)

// Direction of a batch.
type Direction int

const (
	Obfuscate   Direction = C.SQOBFS_OBFUSCATE
	Deobfuscate Direction = C.SQOBFS_DEOBFUSCATE
)

// SaltLen is the salt in front of every datagram: 8 (salamander.go:15) or
// 16 (xplus.go:17).
func (k Kind) SaltLen() int {
	if k == Salamander {
		return C.SQOBFS_SALAMANDER_SALT_LEN
	}
	return C.SQOBFS_XPLUS_SALT_LEN
}

// Error is a negative sqobfs status code.
type Error int

func (e Error) Error() string { return "sqobfs: " + C.GoString(C.sqobfs_strerror(C.int(e))) }

func check(st C.int) error {
	if st != C.SQ_OK {
		return Error(st)
	}
	return nil
}

// ErrClosed is returned by calls on a released Context.
var ErrClosed = errors.New("sqobfs: context closed")

// Context is one GPU (sqobfs_open).  Safe for concurrent use.
type Context struct {
	mu     sync.Mutex
	c      *C.sqobfs_ctx
	refs   int
	device int
	shared bool
}

// Open makes a context of its own on a GPU; Close releases the caller's
// reference.
func Open(device int) (*Context, error) {
	var c *C.sqobfs_ctx
	if err := check(C.sqobfs_open(C.int(device), &c)); err != nil {
		return nil, err
	}
	return &Context{c: c, refs: 1, device: device}, nil
}

var shared struct {
	sync.Mutex
	m map[int]*Context
}

// Shared returns the process's context on a GPU with a new reference (Close
// releases it); it is opened on first use and closed with its last user.
func Shared(device int) (*Context, error) {
	shared.Lock()
	defer shared.Unlock()
	if x := shared.m[device]; x != nil && x.ref() {
		return x, nil
	}
	x, err := Open(device)
	if err != nil {
		return nil, err
	}
	x.shared = true
	if shared.m == nil {
		shared.m = map[int]*Context{}
	}
	shared.m[device] = x
	return x, nil
}

// SetEngineAffinity chooses where the context's packet conn engine runs its
// threads (sqobfs_engine_set_affinity): l3 true (the default) keeps them on
// the CPUs sharing the L3 cache of the goroutine's OS thread that opens the
// first Conn, false leaves them to the scheduler.  Only before that first
// Conn; an error after.
func (x *Context) SetEngineAffinity(l3 bool) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	if x.c == nil {
		return ErrClosed
	}
	mode := C.int(C.SQOBFS_ENGINE_AFFINITY_NONE)
	if l3 {
		mode = C.SQOBFS_ENGINE_AFFINITY_L3
	}
	return check(C.sqobfs_engine_set_affinity(x.c, mode))
}

// SetEngineGroup bounds the coalesced launches of the context's engine
// (sqobfs_engine_set_group): the queued batches of Conns over generic
// PacketConns -- a hop client's conns -- join one launch, at most maxBatches
// of them (0 = 32, 1 = every batch its own launch).  Any time.
func (x *Context) SetEngineGroup(maxBatches int) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	if x.c == nil {
		return ErrClosed
	}
	if maxBatches < 0 {
		return check(C.SQ_EINVAL)
	}
	return check(C.sqobfs_engine_set_group(x.c, C.uint32_t(maxBatches)))
}

// ref takes a reference; false once the context is gone.
func (x *Context) ref() bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	if x.c == nil {
		return false
	}
	x.refs++
	return true
}

// unref drops a reference and closes the C context with the last one.
func (x *Context) unref() {
	x.mu.Lock()
	x.refs--
	last := x.refs == 0 && x.c != nil
	c := x.c
	if last {
		x.c = nil
	}
	x.mu.Unlock()
	if !last {
		return
	}
	if x.shared {
		shared.Lock()
		if shared.m[x.device] == x {
			delete(shared.m, x.device)
		}
		shared.Unlock()
	}
	C.sqobfs_close(c)
}

// Close releases the reference Open or Shared returned.
func (x *Context) Close() { x.unref() }

// Keyring is the copy of the PSK: the `password` captured by
// NewSalamanderConn (salamander.go:19-40) or the `key` of NewXPlusPacketConn
// (xplus.go:19-44) -- on the GPU with its host copy, or host only
// (NewHostKeyring: no GPU needed).
type Keyring struct {
	ctx  *Context // nil: a host keyring
	kr   *C.sqobfs_keyring
	Kind Kind
}

func (x *Context) NewKeyring(kind Kind, psk []byte) (*Keyring, error) {
	if !x.ref() {
		return nil, ErrClosed
	}
	kr, err := newKeyring(x.c, kind, psk)
	if err != nil {
		x.unref()
		return nil, err
	}
	return &Keyring{ctx: x, kr: kr, Kind: kind}, nil
}

// NewHostKeyring makes a keyring that needs no GPU (sqobfs_keyring_create
// with no context): the PSK's hash state on the host, for Conns on the CPU
// path.
func NewHostKeyring(kind Kind, psk []byte) (*Keyring, error) {
	kr, err := newKeyring(nil, kind, psk)
	if err != nil {
		return nil, err
	}
	return &Keyring{kr: kr, Kind: kind}, nil
}

func newKeyring(c *C.sqobfs_ctx, kind Kind, psk []byte) (*C.sqobfs_keyring, error) {
	// a private C copy: the reference's append(password, salt...) can write
	// into the password's spare capacity (SURVEY.md section 5); this never does
	blob := C.malloc(C.size_t(len(psk) + 1))
	defer C.free(blob)
	if len(psk) > 0 {
		C.memcpy(blob, unsafe.Pointer(&psk[0]), C.size_t(len(psk)))
	}
	off := (*C.uint64_t)(C.malloc(8))
	ln := (*C.uint32_t)(C.malloc(4))
	defer C.free(unsafe.Pointer(off))
	defer C.free(unsafe.Pointer(ln))
	*off, *ln = 0, C.uint32_t(len(psk))
	var kr *C.sqobfs_keyring
	if err := check(C.sqobfs_keyring_create(c, C.int(kind), 1, (*C.uint8_t)(blob), off, ln,
		&kr)); err != nil {
		return nil, err
	}
	return kr, nil
}

// Close releases the keyring (sqobfs_keyring_destroy does not block: its
// device memory goes after the launches that used it) and its context
// reference.
func (k *Keyring) Close() {
	if k.kr != nil {
		C.sqobfs_keyring_destroy(k.kr)
		k.kr = nil
		if k.ctx != nil {
			k.ctx.unref()
		}
	}
}

// Slots is a ragged batch of up to Cap datagrams in C memory: a
// page-locked data region of Cap fixed slots of SlotBytes (DMA'd by
// sqobfs_run_host without staging) and the sqobfs_batch descriptor with its
// arrays, all allocated by C.  Go code fills and reads the slots through
// unsafe.Slice views; the C side never sees a Go pointer.  For batches a
// caller assembles itself; Conn uses the engine (sqobfs_pconn) instead.
type Slots struct {
	ctx       *Context
	Cap       int
	SlotBytes int
	data      unsafe.Pointer // sqobfs_host_alloc: Cap*SlotBytes (in) + Cap*SlotBytes (out)
	b         *C.sqobfs_batch
	inOff     []uint64 // views of C arrays
	inLen     []uint32
	outOff    []uint64
	outLen    []uint32
	inCap     []uint32
	salt      []byte
	once      sync.Once
}

func (x *Context) NewSlots(capacity, slotBytes int, saltLen int) (*Slots, error) {
	if capacity <= 0 || slotBytes <= 0 {
		return nil, errors.New("sqobfs: bad slot geometry")
	}
	if !x.ref() {
		return nil, ErrClosed
	}
	s := &Slots{ctx: x, Cap: capacity, SlotBytes: slotBytes}
	if err := check(C.sqobfs_host_alloc(x.c, C.size_t(2*capacity*slotBytes), &s.data)); err != nil {
		x.unref()
		return nil, err
	}
	s.b = (*C.sqobfs_batch)(C.calloc(1, C.size_t(unsafe.Sizeof(C.sqobfs_batch{}))))
	n := C.size_t(capacity)
	io := (*uint64)(C.malloc(8 * n))
	oo := (*uint64)(C.malloc(8 * n))
	il := (*uint32)(C.malloc(4 * n))
	ol := (*uint32)(C.malloc(4 * n))
	ic := (*uint32)(C.malloc(4 * n))
	sl := (*byte)(C.malloc(16 * n)) // malloc alignment >= 16: salts 4-byte aligned
	s.inOff = unsafe.Slice(io, capacity)
	s.outOff = unsafe.Slice(oo, capacity)
	s.inLen = unsafe.Slice(il, capacity)
	s.outLen = unsafe.Slice(ol, capacity)
	s.inCap = unsafe.Slice(ic, capacity)
	s.salt = unsafe.Slice(sl, 16*capacity)
	for i := 0; i < capacity; i++ {
		s.inOff[i] = uint64(i * slotBytes)
		s.outOff[i] = uint64((capacity + i) * slotBytes) // out region after the in region
	}
	base := (*C.uint8_t)(s.data)
	s.b.in = base
	s.b.out = base
	s.b.in_off = (*C.uint64_t)(unsafe.Pointer(io))
	s.b.in_len = (*C.uint32_t)(unsafe.Pointer(il))
	s.b.out_off = (*C.uint64_t)(unsafe.Pointer(oo))
	s.b.out_len = (*C.uint32_t)(unsafe.Pointer(ol))
	s.b.salt = (*C.uint8_t)(unsafe.Pointer(sl))
	// the finalizer only frees C memory; the context stays open until this
	// runs (it holds a reference), so it is never used after sqobfs_close
	runtime.SetFinalizer(s, (*Slots).Free)
	return s, nil
}

// In is input slot i (len SlotBytes); Out is output slot i.
func (s *Slots) In(i int) []byte {
	return unsafe.Slice((*byte)(unsafe.Add(s.data, i*s.SlotBytes)), s.SlotBytes)
}
func (s *Slots) Out(i int) []byte {
	return unsafe.Slice((*byte)(unsafe.Add(s.data, (s.Cap+i)*s.SlotBytes)), s.SlotBytes)
}

// SetLen sets packet i's input length (payload for obfuscate, datagram n for
// deobfuscate); SetCap sets XPlus's read-buffer length len(p) (xplus.go:55).
func (s *Slots) SetLen(i, n int) { s.inLen[i] = uint32(n) }
func (s *Slots) SetCap(i, c int) { s.inCap[i] = uint32(c) }

// Salt is packet i's salt (obfuscate with caller salts).
func (s *Slots) Salt(i, saltLen int) []byte { return s.salt[i*saltLen : (i+1)*saltLen] }

// OutLen is packet i's output length after Run (the reference's return
// value rules, include/sqobfs.h).
func (s *Slots) OutLen(i int) int { return int(s.outLen[i]) }

// Run transforms packets [0, n) in one sqobfs_run_host call (H2D, one
// launch, D2H).  deviceSalt: obfuscate with salts generated on the GPU
// (replaces buf.WriteRandom, salamander.go:60, and math/rand, xplus.go:67-69).
// withCap: XPlus deobfuscate XORs up to SetCap bytes (xplus.go:55).  Output
// bytes are only read up to OutLen, so the output slots are declared
// uninitialised (no copy-in of the output span), and with 16-byte-multiple
// slots as owning their blocks (SQOBFS_FLAG_OUT_BLOCKS; 128-byte multiples:
// their last lines, SQOBFS_FLAG_OUT_LINES).
func (s *Slots) Run(kr *Keyring, dir Direction, n int, deviceSalt, withCap bool) error {
	if n < 0 || n > s.Cap {
		return errors.New("sqobfs: batch larger than its slots")
	}
	s.b.n = C.uint32_t(n)
	s.b.flags = C.SQOBFS_FLAG_OUT_UNINIT
	if s.SlotBytes%128 == 0 {
		// slots of whole 128-byte lines (sqobfs_host_alloc memory is page
		// aligned): the kernel writes every output through to the end of its
		// last line, so no line of the staged copy is written in part
		// (SQOBFS_FLAG_OUT_LINES: ~10 % of the HBM rate on 2,048-byte slots)
		s.b.flags |= C.SQOBFS_FLAG_OUT_LINES
	} else if s.SlotBytes%16 == 0 {
		// every output in a slot of its own: the kernel writes whole blocks
		// (the slot padding is scratch)
		s.b.flags |= C.SQOBFS_FLAG_OUT_BLOCKS
	}
	if dir == Obfuscate && deviceSalt {
		s.b.flags |= C.SQOBFS_FLAG_DEVICE_SALT
	}
	s.b.in_cap = nil
	if withCap {
		s.b.in_cap = (*C.uint32_t)(unsafe.Pointer(&s.inCap[0])) // C memory
	}
	return check(C.sqobfs_run_host(s.ctx.c, kr.kr, C.int(dir), s.b))
}

// Free releases the C memory and the context reference (once; also the
// finalizer's path).
func (s *Slots) Free() {
	s.once.Do(func() {
		runtime.SetFinalizer(s, nil)
		C.free(unsafe.Pointer(s.b.in_off))
		C.free(unsafe.Pointer(s.b.out_off))
		C.free(unsafe.Pointer(s.b.in_len))
		C.free(unsafe.Pointer(s.b.out_len))
		C.free(unsafe.Pointer(&s.inCap[0]))
		C.free(unsafe.Pointer(s.b.salt))
		C.free(unsafe.Pointer(s.b))
		C.sqobfs_host_free(s.ctx.c, s.data)
		s.b = nil
		s.ctx.unref()
	})
}
