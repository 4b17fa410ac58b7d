//go:build linux && sqobfs

package sqobfs

/*
#include <stdlib.h>
#include "sqobfs.h"
*/
import "C"

import (
	"errors"
	"net"
	"net/netip"
	"os"
	"sync"
	"sync/atomic"
	"syscall"
	"time"
	"unsafe"
)

// Options of a Conn.
type Options struct {
	Device    int           // GPU
	NoGPU     bool          // every batch on the CPU path (also the fallback when the GPU cannot be opened)
	Batch     int           // datagrams per launch at most (default 256)
	SlotBytes int           // per-datagram slot (default 2048, hop.go:19)
	Linger    time.Duration // an idle engine waits this long for a batch to grow (default 0)
	Pump      bool          // move datagrams through the wrapped conn even when it is a *net.UDPConn
	NoOffload bool          // socket mode: no UDP GSO on send / GRO on receive
	// CPUMax: batches costing at most this (payload bytes + 1 KiB per
	// datagram) run on the CPU path, not a launch (0: the engine's measured
	// break-even, launch round trip x CPU-path rate -- and, while the
	// engine's traffic would keep more than a tenth of a core busy on the
	// CPU path, a batch of more than 64 datagrams launches, waiting without
	// polling, when that costs the host less CPU; < 0: always launch)
	CPUMax int
	// InlineGap: a WriteTo made while the engine is idle, at least this long
	// after the previous one, is obfuscated and sent on the calling goroutine
	// and returns its own send error, as the reference's (0: 100 us; < 0: never)
	InlineGap time.Duration
}

// Conn is the obfuscating net.PacketConn of SalamanderPacketConn
// (hysteria2/salamander.go:19-74) and XPlusPacketConn (hysteria/xplus.go:39-79)
// with the byte work batched onto the GPU by the engine of include/sqobfs.h
// (sqobfs_pconn_*; its behaviour is tested natively by tests/cpp/test_pconn.c):
//
//   - WriteTo (salamander.go:57-70, xplus.go:62-75) copies p into the transmit
//     batch being filled and returns (p is never mutated, also not by the
//     vectorised variants, unlike salamander.go:85-87); the engine obfuscates
//     the batch in ONE launch (salts from the GPU's generator) as soon as it
//     is idle and sends it, and a send error is returned by the next WriteTo.
//     A WriteTo made while the engine is idle (a handshake, an ACK) is
//     instead obfuscated on the CPU and sent by the calling goroutine, and
//     returns its own send error, as the reference's (Options.InlineGap).
//   - Small batches run on the CPU path (Options.CPUMax), bulk traffic on the
//     GPU (the engine's load mode, sqobfs_engine_info.loaded); with no usable GPU
//     every batch does, so NewConn does not fail for want of a device, and a
//     failed launch moves the engine to the CPU instead of failing the Conn.
//   - ReadFrom (salamander.go:42-55, xplus.go:46-60) returns the next datagram
//     of a batch the engine received and de-obfuscated in ONE launch, with
//     the reference's lengths: for a datagram of w bytes and m = min(w,
//     len(p)), Salamander returns the m raw bytes if m <= 8, else the first
//     m - 8 payload bytes; XPlus returns 0 if m < 16, else m - 16 bytes.  Not
//     reproduced: XPlus's ReadFrom also XORs p past the returned length up to
//     len(p) (xplus.go:55), bytes no caller reads.
//   - SetDeadline / SetReadDeadline / SetWriteDeadline apply to these calls
//     (a blocked ReadFrom returns os.ErrDeadlineExceeded when its deadline
//     passes), not to the wrapped conn, which the engine drives itself.
//   - Close sends what was written, then fails every blocked call with
//     net.ErrClosed and frees the engine.
//
// When the wrapped conn is a *net.UDPConn the engine works its socket with
// recvmmsg / sendmmsg (socket mode, SURVEY.md 8(f) rank 1).  Any other
// PacketConn (HopPacketConn, a test double) is driven by two goroutines
// that feed the engine (pump mode).
type Conn struct {
	net.PacketConn
	kind Kind
	ctx  *Context // nil: no GPU, every batch on the CPU path
	kr   *Keyring
	opt  Options

	mu     sync.RWMutex // RLock: a call on pc is in progress; Lock: pc is freed
	pc     *C.sqobfs_pconn
	closed atomic.Bool
	once   sync.Once
	cerr   error

	socket bool
	wg     sync.WaitGroup // pump goroutines
	addrMu sync.Mutex     // pump: the net.Addr of every datagram in flight
	addrs  map[uint64]net.Addr
	tag    uint64
	errMu  sync.Mutex
	txErr  error // pump: the wrapped conn's write error, for the next WriteTo
	rxErr  error // pump: the wrapped conn's read error (SQ_EIO)
}

func (c *Conn) setErr(dst *error, e error) {
	c.errMu.Lock()
	*dst = e
	c.errMu.Unlock()
}

func (c *Conn) getErr(src *error, clear bool) error {
	c.errMu.Lock()
	defer c.errMu.Unlock()
	e := *src
	if clear {
		*src = nil
	}
	return e
}

// NewConn wraps conn; psk is the password (Salamander) or key (XPlus).  It
// uses the GPU when one can be opened and the CPU path otherwise, so it
// fails only when the process is out of memory or threads.
func NewConn(conn net.PacketConn, kind Kind, psk []byte, opt Options) (*Conn, error) {
	if !opt.NoGPU {
		if c, err := newConn(conn, kind, psk, opt, true); err == nil {
			return c, nil
		}
	}
	return newConn(conn, kind, psk, opt, false)
}

func newConn(conn net.PacketConn, kind Kind, psk []byte, opt Options, gpu bool) (*Conn, error) {
	var ctx *Context
	var kr *Keyring
	var err error
	if gpu {
		if ctx, err = Shared(opt.Device); err != nil {
			return nil, err
		}
		kr, err = ctx.NewKeyring(kind, psk)
	} else {
		kr, err = NewHostKeyring(kind, psk)
	}
	if err != nil {
		if ctx != nil {
			ctx.Close()
		}
		return nil, err
	}
	c := &Conn{PacketConn: conn, kind: kind, ctx: ctx, kr: kr, opt: opt}
	var cc *C.sqobfs_ctx
	if ctx != nil {
		cc = ctx.c
	}
	var o C.sqobfs_pconn_opts
	o.batch = C.uint32_t(opt.Batch)
	o.slot_bytes = C.uint32_t(opt.SlotBytes)
	o.linger_us = C.uint32_t(opt.Linger / time.Microsecond)
	switch {
	case opt.CPUMax < 0:
		o.cpu_max = C.SQOBFS_PCONN_NEVER
	case opt.CPUMax > 0:
		o.cpu_max = C.uint32_t(opt.CPUMax)
	}
	switch {
	case opt.InlineGap < 0:
		o.inline_gap_us = C.SQOBFS_PCONN_NEVER
	case opt.InlineGap > 0:
		o.inline_gap_us = C.uint32_t((opt.InlineGap + time.Microsecond - 1) / time.Microsecond)
	}
	if !opt.NoOffload {
		// UDP_SEGMENT / UDP_GRO, as quic-go uses on its own sockets
		// (sys_conn_oob.go); the engine falls back if the socket refuses
		o.flags = C.SQOBFS_UDP_TX_GSO | C.SQOBFS_UDP_RX_GRO
	}
	st := C.int(C.SQ_EINVAL)
	if uc, ok := conn.(*net.UDPConn); ok && !opt.Pump {
		// socket mode: the engine dup()s the fd inside Control, so it never
		// uses a descriptor the runtime may have closed
		if raw, e := uc.SyscallConn(); e == nil {
			_ = raw.Control(func(fd uintptr) {
				st = C.sqobfs_pconn_open(cc, kr.kr, C.int(fd), &o, &c.pc)
			})
			c.socket = st == C.SQ_OK
		}
	}
	if !c.socket {
		c.addrs = map[uint64]net.Addr{}
		o.flags = 0 // offloads are socket mode's
		st = C.sqobfs_pconn_open(cc, kr.kr, -1, &o, &c.pc)
	}
	if err := check(st); err != nil {
		kr.Close()
		if ctx != nil {
			ctx.Close()
		}
		return nil, err
	}
	if !c.socket {
		c.wg.Add(2)
		go c.pumpRx()
		go c.pumpTx()
	}
	return c, nil
}

// ---- errors

func (c *Conn) opErr(op string, st C.int, addr net.Addr) error {
	var e error
	switch {
	case st == C.SQ_ETIMEDOUT:
		e = os.ErrDeadlineExceeded
	case st == C.SQ_ECLOSED:
		e = net.ErrClosed
	case st == C.SQ_EIO:
		if x := c.getErr(&c.rxErr, false); x != nil {
			return x // the wrapped conn's own error, verbatim (salamander.go:43-46)
		}
		e = Error(st)
	case st <= -1000:
		e = os.NewSyscallError(op, syscall.Errno(-1000-int(st)))
	default:
		e = Error(st)
	}
	return &net.OpError{Op: op, Net: "udp", Source: c.LocalAddr(), Addr: addr, Err: e}
}

// ---- addresses

func toCAddr(a net.Addr) (C.sqobfs_addr, bool) {
	var ca C.sqobfs_addr
	var ap netip.AddrPort
	switch x := a.(type) {
	case *net.UDPAddr:
		ap = x.AddrPort()
	default:
		p, err := netip.ParseAddrPort(a.String())
		if err != nil {
			return ca, false
		}
		ap = p
	}
	ip := ap.Addr()
	ca.port = C.uint16_t(ap.Port())
	if ip.Is4() || ip.Is4In6() {
		ca.family = C.uint16_t(syscall.AF_INET)
		b := ip.Unmap().As4()
		for i := 0; i < 4; i++ {
			ca.addr[i] = C.uint8_t(b[i])
		}
	} else {
		ca.family = C.uint16_t(syscall.AF_INET6)
		b := ip.As16()
		for i := 0; i < 16; i++ {
			ca.addr[i] = C.uint8_t(b[i])
		}
		if z := ip.Zone(); z != "" {
			if ifi, err := net.InterfaceByName(z); err == nil {
				ca.scope_id = C.uint32_t(ifi.Index)
			}
		}
	}
	return ca, true
}

func fromCAddr(ca *C.sqobfs_addr) net.Addr {
	if ca.family == C.uint16_t(syscall.AF_INET6) {
		var b [16]byte
		for i := range b {
			b[i] = byte(ca.addr[i])
		}
		ua := &net.UDPAddr{IP: net.IP(b[:]), Port: int(ca.port)}
		if ca.scope_id != 0 {
			if ifi, err := net.InterfaceByIndex(int(ca.scope_id)); err == nil {
				ua.Zone = ifi.Name
			}
		}
		return ua
	}
	return &net.UDPAddr{IP: net.IPv4(byte(ca.addr[0]), byte(ca.addr[1]), byte(ca.addr[2]),
		byte(ca.addr[3])), Port: int(ca.port)}
}

func (c *Conn) putAddr(a net.Addr) uint64 {
	c.addrMu.Lock()
	c.tag++
	t := c.tag
	if c.addrs != nil { // (nil after Close)
		c.addrs[t] = a
	}
	c.addrMu.Unlock()
	return t
}

func (c *Conn) takeAddr(t uint64) net.Addr {
	c.addrMu.Lock()
	a := c.addrs[t]
	delete(c.addrs, t)
	c.addrMu.Unlock()
	return a
}

func bytePtr(p []byte) *C.uint8_t {
	if len(p) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&p[0]))
}

// ---- net.PacketConn

// WriteTo returns len(p) for Salamander (salamander.go:69) and len(p) + 16
// for XPlus (xplus.go:74 returns the inner write's n).
func (c *Conn) WriteTo(p []byte, addr net.Addr) (int, error) {
	if e := c.getErr(&c.txErr, true); e != nil {
		return 0, e
	}
	c.mu.RLock()
	defer c.mu.RUnlock()
	if c.pc == nil {
		return 0, c.opErr("write", C.SQ_ECLOSED, addr)
	}
	var st C.int
	if c.socket {
		ca, ok := toCAddr(addr)
		if !ok {
			return 0, &net.OpError{Op: "write", Net: "udp", Addr: addr,
				Err: errors.New("sqobfs: not a UDP address")}
		}
		st = C.sqobfs_pconn_write(c.pc, bytePtr(p), C.uint32_t(len(p)), &ca, 0)
	} else {
		t := c.putAddr(addr)
		st = C.sqobfs_pconn_write(c.pc, bytePtr(p), C.uint32_t(len(p)), nil, C.uint64_t(t))
		if st != C.SQ_OK {
			c.takeAddr(t)
		}
	}
	if st != C.SQ_OK {
		return 0, c.opErr("write", st, addr)
	}
	if c.kind == XPlus {
		return len(p) + XPlus.SaltLen(), nil
	}
	return len(p), nil
}

func (c *Conn) ReadFrom(p []byte) (int, net.Addr, error) {
	c.mu.RLock()
	defer c.mu.RUnlock()
	if c.pc == nil {
		return 0, nil, c.opErr("read", C.SQ_ECLOSED, nil)
	}
	var n C.uint32_t
	var from C.sqobfs_addr
	var tag C.uint64_t
	st := C.sqobfs_pconn_read(c.pc, bytePtr(p), C.uint32_t(len(p)), &n, &from, &tag)
	if st != C.SQ_OK {
		return 0, nil, c.opErr("read", st, nil)
	}
	if c.socket {
		return int(n), fromCAddr(&from), nil
	}
	return int(n), c.takeAddr(uint64(tag)), nil
}

func deadlineNs(t time.Time) C.int64_t {
	if t.IsZero() {
		return 0
	}
	if ns := t.UnixNano(); ns > 0 {
		return C.int64_t(ns)
	}
	return 1 // before the epoch: passed
}

func (c *Conn) setDeadline(which C.uint32_t, t time.Time) error {
	c.mu.RLock()
	defer c.mu.RUnlock()
	if c.pc == nil {
		return c.opErr("set", C.SQ_ECLOSED, nil)
	}
	return check(C.sqobfs_pconn_set_deadline(c.pc, which, deadlineNs(t)))
}

func (c *Conn) SetDeadline(t time.Time) error {
	return c.setDeadline(C.SQOBFS_PCONN_READ|C.SQOBFS_PCONN_WRITE, t)
}
func (c *Conn) SetReadDeadline(t time.Time) error  { return c.setDeadline(C.SQOBFS_PCONN_READ, t) }
func (c *Conn) SetWriteDeadline(t time.Time) error { return c.setDeadline(C.SQOBFS_PCONN_WRITE, t) }

// Upstream is the sing unwrap convention (salamander.go:72-74, xplus.go:77-79).
func (c *Conn) Upstream() any { return c.PacketConn }

// Close: writes already made are sent (bounded, 200 ms), blocked calls fail
// with net.ErrClosed, the wrapped conn is closed, then the engine, the
// keyring and the context reference are released.
func (c *Conn) Close() error {
	c.once.Do(func() {
		c.closed.Store(true)
		c.mu.RLock()
		C.sqobfs_pconn_shutdown(c.pc) // wakes every blocked call, ends the workers
		c.mu.RUnlock()
		c.cerr = c.PacketConn.Close() // ends the pump reader's inner ReadFrom
		c.wg.Wait()
		c.mu.Lock() // no call on pc is in progress past this point
		C.sqobfs_pconn_close(c.pc)
		c.pc = nil
		c.mu.Unlock()
		// pump mode: addresses of datagrams that never reached a ReadFrom or
		// the wrapped conn (queued at Close, or lost with a failed launch)
		c.addrMu.Lock()
		c.addrs = nil
		c.addrMu.Unlock()
		c.kr.Close()
		if c.ctx != nil {
			c.ctx.Close()
		}
	})
	return c.cerr
}

// ---- pump mode: the wrapped conn's I/O on two goroutines

func (c *Conn) pumpRx() {
	defer c.wg.Done()
	buf := make([]byte, 65536) // a whole UDP datagram; the engine cuts to its slot
	for {
		n, addr, err := c.PacketConn.ReadFrom(buf)
		if err != nil {
			if c.closed.Load() {
				return
			}
			c.setErr(&c.rxErr, err)
			// a timeout or an ICMP-reported refusal is per call: the next read
			// works; anything else ends the receive side
			var ne net.Error
			once := errors.As(err, &ne) && ne.Timeout() ||
				errors.Is(err, syscall.ECONNREFUSED)
			c.mu.RLock()
			_ = C.sqobfs_pconn_rx_fail(c.pc, C.SQ_EIO, boolInt(once))
			c.mu.RUnlock()
			if !once {
				return
			}
			continue
		}
		t := c.putAddr(addr)
		c.mu.RLock()
		st := C.sqobfs_pconn_rx_push(c.pc, bytePtr(buf[:n]), C.uint32_t(n), nil, C.uint64_t(t))
		c.mu.RUnlock()
		if st != C.SQ_OK {
			c.takeAddr(t)
			if st == C.SQ_ECLOSED {
				return
			}
		}
	}
}

func (c *Conn) pumpTx() {
	defer c.wg.Done()
	for {
		var v C.sqobfs_pconn_tx
		c.mu.RLock()
		st := C.sqobfs_pconn_tx_take(c.pc, -1, &v)
		c.mu.RUnlock()
		if st != C.SQ_OK {
			return // SQ_ECLOSED: shut down
		}
		n := int(v.count)
		offs := unsafe.Slice((*uint64)(unsafe.Pointer(v.off)), n)
		lens := unsafe.Slice((*uint32)(unsafe.Pointer(v.len)), n)
		tags := unsafe.Slice((*uint64)(unsafe.Pointer(v.tag)), n)
		for i := 0; i < n; i++ {
			wire := unsafe.Slice((*byte)(unsafe.Add(unsafe.Pointer(v.base), offs[i])), lens[i])
			if _, err := c.PacketConn.WriteTo(wire, c.takeAddr(tags[i])); err != nil {
				c.setErr(&c.txErr, err)
			}
		}
		c.mu.RLock()
		_ = C.sqobfs_pconn_tx_done(c.pc)
		c.mu.RUnlock()
	}
}

func boolInt(b bool) C.int {
	if b {
		return 1
	}
	return 0
}
