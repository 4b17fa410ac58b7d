//go:build linux && sqobfs

package sqobfs

import (
	"errors"
	"net"
	"os"
	"sync"
	"sync/atomic"
	"time"
)

// Options of a Conn.
type Options struct {
	Device    int           // GPU
	Batch     int           // datagrams per launch (default 256)
	SlotBytes int           // per-datagram slot (default 2048, hop.go:19)
	Linger    time.Duration // longest a datagram waits for its batch (default 50us)
}

func (o *Options) defaults() {
	if o.Batch <= 0 {
		o.Batch = 256
	}
	if o.SlotBytes <= 0 {
		o.SlotBytes = 2048
	}
	if o.Linger <= 0 {
		o.Linger = 50 * time.Microsecond
	}
}

// Conn is the obfuscating net.PacketConn of SalamanderPacketConn
// (hysteria2/salamander.go:19-74) and XPlusPacketConn (hysteria/xplus.go:39-79)
// with the byte work batched onto the GPU:
//
//   - WriteTo (salamander.go:57-70, xplus.go:62-75) copies the payload into
//     the transmit batch being filled and returns; a flusher obfuscates the
//     batch in ONE launch (salts generated on the GPU) as soon as it is full
//     or Linger after its first datagram, then writes the datagrams to the
//     wrapped conn in order.  An error of those writes is returned by the
//     next WriteTo (UDP is best-effort; quic-go reuses p after WriteTo, so p
//     is always copied).
//   - ReadFrom (salamander.go:42-55, xplus.go:46-60) is fed by a reader
//     goroutine that drains the wrapped conn into receive batches and
//     de-obfuscates each batch in ONE launch.  Returned lengths follow the
//     reference exactly (Salamander n <= 8 returns the raw datagram; XPlus
//     n < 16 returns 0).  Not reproduced: XPlus's ReadFrom also XORs p past
//     the returned length up to len(p) (xplus.go:55), garbage bytes no
//     caller reads; the C ABI reproduces it (in_cap) when asked.
type Conn struct {
	net.PacketConn
	kind Kind
	ctx  *Context
	kr   *Keyring
	opt  Options

	txMu    sync.Mutex
	txFill  *Slots
	txAddr  []net.Addr
	txN     int
	txFirst time.Time
	txFree  chan *Slots
	txWork  chan txJob
	txErr   atomic.Value // error

	rx     chan rxItem
	rxErr  atomic.Value // error
	closed chan struct{}
	once   sync.Once
	wg     sync.WaitGroup
}

type txJob struct {
	s    *Slots
	addr []net.Addr
	n    int
}

type rxItem struct {
	s    *rxBatch
	i    int
	addr net.Addr
}

type rxBatch struct {
	s    *Slots
	left int32 // datagrams not yet consumed
	free chan *rxBatch
}

// NewConn wraps conn; psk is the password (Salamander) or key (XPlus).
func NewConn(conn net.PacketConn, kind Kind, psk []byte, opt Options) (*Conn, error) {
	opt.defaults()
	ctx, err := Open(opt.Device)
	if err != nil {
		return nil, err
	}
	kr, err := ctx.NewKeyring(kind, psk)
	if err != nil {
		ctx.Close()
		return nil, err
	}
	c := &Conn{PacketConn: conn, kind: kind, ctx: ctx, kr: kr, opt: opt,
		txFree: make(chan *Slots, 2), txWork: make(chan txJob, 2),
		rx: make(chan rxItem, 4*opt.Batch), closed: make(chan struct{})}
	for i := 0; i < 2; i++ {
		s, err := ctx.NewSlots(opt.Batch, opt.SlotBytes, kind.SaltLen())
		if err != nil {
			c.free()
			return nil, err
		}
		c.txFree <- s
	}
	rxFree := make(chan *rxBatch, 3)
	for i := 0; i < 3; i++ {
		s, err := ctx.NewSlots(opt.Batch, opt.SlotBytes, kind.SaltLen())
		if err != nil {
			c.free()
			return nil, err
		}
		rxFree <- &rxBatch{s: s, free: rxFree}
	}
	c.wg.Add(2)
	go c.flusher()
	go c.reader(rxFree)
	return c, nil
}

// ---- transmit

func (c *Conn) WriteTo(p []byte, addr net.Addr) (int, error) {
	if e, _ := c.txErr.Load().(error); e != nil {
		return 0, e
	}
	S := c.kind.SaltLen()
	if len(p)+S > c.opt.SlotBytes {
		return 0, errors.New("sqobfs: datagram larger than the slot")
	}
	c.txMu.Lock()
	if c.txFill == nil {
		select {
		case c.txFill = <-c.txFree:
		case <-c.closed:
			c.txMu.Unlock()
			return 0, net.ErrClosed
		}
		c.txN = 0
		c.txAddr = c.txAddr[:0]
		c.txFirst = time.Now()
		go c.lingerKick(c.txFill)
	}
	i := c.txN
	c.txFill.SetLen(i, copy(c.txFill.In(i), p))
	c.txAddr = append(c.txAddr, addr)
	c.txN++
	if c.txN == c.txFill.Cap {
		c.handOff()
	}
	c.txMu.Unlock()
	if c.kind == XPlus {
		return len(p) + S, nil // xplus.go:74 returns the inner write's n
	}
	return len(p), nil // salamander.go:69
}

// handOff passes the filling batch to the flusher (txMu held).
func (c *Conn) handOff() {
	c.txWork <- txJob{s: c.txFill, addr: append([]net.Addr(nil), c.txAddr...), n: c.txN}
	c.txFill = nil
}

// lingerKick flushes a partly filled batch Linger after its first datagram.
func (c *Conn) lingerKick(s *Slots) {
	t := time.NewTimer(c.opt.Linger)
	defer t.Stop()
	select {
	case <-t.C:
	case <-c.closed:
		return
	}
	c.txMu.Lock()
	if c.txFill == s && c.txN > 0 {
		c.handOff()
	}
	c.txMu.Unlock()
}

func (c *Conn) flusher() {
	defer c.wg.Done()
	for {
		var j txJob
		select {
		case j = <-c.txWork:
		case <-c.closed:
			return
		}
		err := j.s.Run(c.kr, Obfuscate, j.n, true, false)
		for i := 0; i < j.n && err == nil; i++ {
			_, err = c.PacketConn.WriteTo(j.s.Out(i)[:j.s.OutLen(i)], j.addr[i])
		}
		if err != nil {
			c.txErr.Store(err)
		}
		c.txFree <- j.s
	}
}

// ---- receive

func (c *Conn) reader(free chan *rxBatch) {
	defer c.wg.Done()
	for {
		var rb *rxBatch
		select {
		case rb = <-free:
		case <-c.closed:
			return
		}
		s := rb.s
		addrs := make([]net.Addr, 0, s.Cap)
		n := 0
		for n < s.Cap {
			if n == 1 { // batch what is already queued, for at most Linger
				_ = c.PacketConn.SetReadDeadline(time.Now().Add(c.opt.Linger))
			}
			m, addr, err := c.PacketConn.ReadFrom(s.In(n))
			if err != nil {
				if n > 0 && errors.Is(err, os.ErrDeadlineExceeded) {
					break
				}
				c.rxErr.Store(err)
				close(c.rx)
				return
			}
			s.SetLen(n, m)
			addrs = append(addrs, addr)
			n++
		}
		_ = c.PacketConn.SetReadDeadline(time.Time{})
		if err := s.Run(c.kr, Deobfuscate, n, false, false); err != nil {
			c.rxErr.Store(err)
			close(c.rx)
			return
		}
		rb.left = int32(n)
		for i := 0; i < n; i++ {
			c.rx <- rxItem{s: rb, i: i, addr: addrs[i]}
		}
	}
}

func (c *Conn) ReadFrom(p []byte) (int, net.Addr, error) {
	it, ok := <-c.rx
	if !ok {
		if e, _ := c.rxErr.Load().(error); e != nil {
			return 0, nil, e
		}
		return 0, nil, net.ErrClosed
	}
	n := copy(p, it.s.s.Out(it.i)[:it.s.s.OutLen(it.i)])
	if atomic.AddInt32(&it.s.left, -1) == 0 {
		it.s.free <- it.s
	}
	return n, it.addr, nil
}

// Upstream is the sing unwrap convention (salamander.go:72-74, xplus.go:77-79).
func (c *Conn) Upstream() any { return c.PacketConn }

func (c *Conn) Close() error {
	c.once.Do(func() { close(c.closed) })
	err := c.PacketConn.Close()
	c.wg.Wait()
	c.free()
	return err
}

func (c *Conn) free() {
	for {
		select {
		case s := <-c.txFree:
			s.Free()
			continue
		default:
		}
		break
	}
	c.kr.Close()
	c.ctx.Close()
}
