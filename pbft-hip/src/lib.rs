//! pbft-hip: the MI355X batch verifier that gates PBFT's Prepare / Commit quorums
//! (BASELINE.json north_star), as the crate ameya-deshmukh/pbft would depend on.
//!
//! * [`BatchVerifier`]: the trait of SURVEY.md §8(b) -- non-blocking `submit` + `poll`
//!   (fits `NetworkBehaviour::poll`, /root/reference/src/behavior.rs:416-426) and a
//!   blocking `verify`.  An invalid signature is a 0 bit, never an error (the reference
//!   panics through `.unwrap()`, src/behavior.rs:345, :371).
//! * [`GpuVerifier`]: the HIP implementation (libpbft_verify.so, gfx950).
//! * [`CpuVerifier`] (feature `cpu`): ed25519-dalek 1.0.1 `PublicKey::verify_strict` per
//!   signature -- the reference's own crypto (libp2p-core 0.31.1 -> ed25519-dalek 1.0.1,
//!   Cargo.lock:668-679).  UNTESTED: there is no Rust toolchain in the build image, so this
//!   implementation has never been compiled or run; the GPU path's bit-exactness is established
//!   against the repository's C and Python restatements of verify_strict (tests/golden), not
//!   against this code.
//! * [`Replica`]: the native round batcher + quorum state machine
//!   (include/pbft_replica.h) that replaces `validate_prepare` / `validate_commit`
//!   (src/behavior.rs:159-195) and keys votes by the authenticated peer
//!   (src/behavior.rs:346, :380); any `BatchVerifier` can back it.
//! * [`key_from_peer_id`]: libp2p PeerId -> Ed25519 key (src/main.rs:39-40).
//!
//! NOT COMPILED IN THIS REPOSITORY: the build image has no Rust toolchain.  Every C entry
//! point used here is exercised through ctypes by tests/ (CPU) and tests/ -m gpu (MI355X).
use std::ffi::CStr;
use std::fmt;
use std::marker::PhantomData;
use std::os::raw::{c_int, c_void};
use std::ptr;

pub mod ffi;

/// The 85-byte signed envelope: "PBFT" || kind || view LE || seq LE || digest[64].
pub type Envelope = [u8; ffi::PBFT_ENVELOPE_BYTES];

#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

impl fmt::Display for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "pbft-hip error {}: {}", self.code, self.message)
    }
}
impl std::error::Error for Error {}

pub type Result<T> = std::result::Result<T, Error>;

fn check(rc: c_int) -> Result<c_int> {
    if rc >= 0 {
        return Ok(rc);
    }
    let message = unsafe { CStr::from_ptr(ffi::pbft_last_error()) }.to_string_lossy().into_owned();
    Err(Error { code: rc, message })
}

/// Encode the signed envelope (the bytes every Prepare / Commit / PrePrepare signature covers).
pub fn envelope(kind: u8, view: u64, seq: u64, digest: &[u8; 64]) -> Envelope {
    let mut out = [0u8; ffi::PBFT_ENVELOPE_BYTES];
    unsafe { ffi::pbft_envelope(out.as_mut_ptr(), kind, view, seq, digest.as_ptr()) };
    out
}

/// Struct-of-arrays batch of one or more (view, seq) round windows.
#[derive(Clone, Default)]
pub struct SigBatch {
    pub r: Vec<[u8; 32]>,
    pub s: Vec<[u8; 32]>,
    pub key_idx: Vec<u16>,
    pub msg: Vec<Envelope>,
}

impl SigBatch {
    pub fn push(&mut self, key_idx: u16, envelope: Envelope, sig: &[u8; 64]) {
        let mut r = [0u8; 32];
        let mut s = [0u8; 32];
        r.copy_from_slice(&sig[..32]);
        s.copy_from_slice(&sig[32..]);
        self.r.push(r);
        self.s.push(s);
        self.key_idx.push(key_idx);
        self.msg.push(envelope);
    }
    pub fn len(&self) -> usize {
        self.r.len()
    }
    pub fn is_empty(&self) -> bool {
        self.r.is_empty()
    }
}

/// Votes form of a round batch: signature i signs `envelopes[env_idx[i]]` (a window's Prepares / Commits
/// all sign the same (kind, view, seq, digest) envelope), 70 bytes per signature over PCIe instead of 151.
#[derive(Clone, Default)]
pub struct VotesBatch {
    pub r: Vec<[u8; 32]>,
    pub s: Vec<[u8; 32]>,
    pub key_idx: Vec<u16>,
    pub env_idx: Vec<u32>,
    pub envelopes: Vec<Envelope>,
}

impl VotesBatch {
    pub fn len(&self) -> usize {
        self.r.len()
    }
    pub fn is_empty(&self) -> bool {
        self.r.is_empty()
    }
    /// Err(PBFT_EINVAL) unless `s`, `key_idx` and `env_idx` have one entry per signature (`r`).
    pub fn check_columns(&self) -> Result<()> {
        let n = self.r.len();
        if self.s.len() != n || self.key_idx.len() != n || self.env_idx.len() != n {
            return Err(Error { code: ffi::PBFT_EINVAL, message: "VotesBatch: column lengths differ".into() });
        }
        Ok(())
    }
    /// The per-signature form (every signature carrying its own envelope), for verifiers without a votes form.
    pub fn to_sig_batch(&self) -> Result<SigBatch> {
        self.check_columns()?;
        let mut b = SigBatch::default();
        for i in 0..self.len() {
            let e = self.envelopes.get(self.env_idx[i] as usize).copied().unwrap_or([0u8; ffi::PBFT_ENVELOPE_BYTES]);
            let mut sig = [0u8; 64];
            sig[..32].copy_from_slice(&self.r[i]);
            sig[32..].copy_from_slice(&self.s[i]);
            // an out-of-range envelope index is a 0 bit: an out-of-range key index gives the same
            let k = if (self.env_idx[i] as usize) < self.envelopes.len() { self.key_idx[i] } else { u16::MAX };
            b.push(k, e, &sig);
        }
        Ok(b)
    }
}

/// Accept bits, LSB-first in u64 words; bits past the batch length are 0.
#[derive(Clone, Debug, Default, PartialEq, Eq)]
pub struct Bitmap(pub Vec<u64>);

impl Bitmap {
    pub fn zeros(n: usize) -> Self {
        Bitmap(vec![0u64; (n + 63) / 64])
    }
    pub fn get(&self, i: usize) -> bool {
        (self.0[i / 64] >> (i % 64)) & 1 == 1
    }
    pub fn set(&mut self, i: usize) {
        self.0[i / 64] |= 1u64 << (i % 64);
    }
}

/// Handle of one submitted batch.
#[derive(Debug, PartialEq, Eq)]
pub struct Ticket(pub u64);

/// the verifier behind the round batcher.
pub trait BatchVerifier {
    /// Install the replica key set (libp2p identity keys of network.json's nodes);
    /// returns key_ok per key (false: bad encoding or small order -> every signature under it is 0).
    fn set_keys(&mut self, keys: &[[u8; 32]]) -> Result<Vec<bool>>;
    /// Non-blocking: enqueue the batch.
    fn submit(&mut self, batch: SigBatch) -> Result<Ticket>;
    /// Ok(Some(bitmap)) once the batch is verified, Ok(None) while it runs.
    fn poll(&mut self, ticket: &Ticket) -> Result<Option<Bitmap>>;
    /// Blocking verify.
    fn verify(&mut self, batch: SigBatch) -> Result<Bitmap> {
        let t = self.submit(batch)?;
        loop {
            if let Some(bm) = self.poll(&t)? {
                return Ok(bm);
            }
            std::thread::yield_now();
        }
    }
}

/// One HIP context (one MI355X).  Not `Sync`: one per thread; `try_clone` for more streams.
pub struct GpuVerifier {
    ctx: *mut ffi::pbft_ctx,
    // the library copies pageable batches into its pinned staging before the DMA, so only the output
    // bitmap (written when the batch completes) has to outlive the call
    inflight: Option<(u64, Bitmap)>,
    next: u64,
}

unsafe impl Send for GpuVerifier {}

impl GpuVerifier {
    pub fn new(device: i32) -> Result<Self> {
        let mut ctx = ptr::null_mut();
        check(unsafe { ffi::pbft_verify_ctx_create(device, &mut ctx) })?;
        Ok(GpuVerifier { ctx, inflight: None, next: 0 })
    }
    /// Non-blocking votes-form submit (pbft_verify_votes_async); complete it with `poll`.
    pub fn submit_votes(&mut self, batch: &VotesBatch) -> Result<Ticket> {
        if self.inflight.is_some() {
            return Err(Error { code: ffi::PBFT_EBUSY, message: "one batch in flight per context".into() });
        }
        batch.check_columns()?; // the C side reads n entries of every column
        let n = batch.len();
        let mut out = Bitmap::zeros(n);
        check(unsafe {
            ffi::pbft_verify_votes_async(self.ctx, batch.r.as_ptr() as *const u8, batch.s.as_ptr() as *const u8,
                                         batch.key_idx.as_ptr(), batch.env_idx.as_ptr(),
                                         batch.envelopes.as_ptr() as *const u8, batch.envelopes.len() as u32,
                                         n as u64, out.0.as_mut_ptr())
        })?;
        self.next += 1;
        self.inflight = Some((self.next, out));
        Ok(Ticket(self.next))
    }
    /// Another context on the same GPU sharing this one's tables (own HIP stream).
    pub fn try_clone(&self) -> Result<Self> {
        let mut ctx = ptr::null_mut();
        check(unsafe { ffi::pbft_verify_ctx_clone(self.ctx, &mut ctx) })?;
        Ok(GpuVerifier { ctx, inflight: None, next: 0 })
    }
    /// Replace keys `idx[i]` of the installed set by `keys[i]` in place (only their tables are rebuilt): a peer
    /// admitted later (Pbft::add_peer, src/behavior.rs:45-61) fills the slot its replica id reserves.
    /// Returns key_ok of the new keys.
    pub fn update_keys(&mut self, idx: &[u32], keys: &[[u8; 32]]) -> Result<Vec<bool>> {
        if idx.len() != keys.len() {
            return Err(Error { code: ffi::PBFT_EINVAL, message: "update_keys: idx and keys lengths differ".into() });
        }
        let mut ok = vec![0u8; keys.len()];
        check(unsafe {
            ffi::pbft_verify_update_keys(self.ctx, idx.as_ptr(), keys.as_ptr() as *const u8, keys.len() as u32,
                                         ok.as_mut_ptr())
        })?;
        Ok(ok.into_iter().map(|b| b == 1).collect())
    }
    /// Where the last set_keys / update_keys spent its time.
    pub fn key_stats(&self) -> ffi::pbft_key_stats {
        let mut s = ffi::pbft_key_stats::default();
        unsafe { ffi::pbft_verify_key_stats(self.ctx, &mut s) };
        s
    }
    pub fn set_option(&mut self, option: i32, value: u64) -> Result<()> {
        check(unsafe { ffi::pbft_verify_set_option(self.ctx, option, value) }).map(|_| ())
    }
    /// Blake2b-512 request digests (src/message.rs:209-212), one per item.
    pub fn blake2b512(&mut self, items: &[&[u8]]) -> Result<Vec<[u8; 64]>> {
        let (data, offs, lens) = pack(items);
        let mut out = vec![[0u8; 64]; items.len()];
        check(unsafe {
            ffi::pbft_digest_blake2b512(self.ctx, data.as_ptr(), offs.as_ptr(), lens.as_ptr(), items.len() as u64,
                                        out.as_mut_ptr() as *mut u8)
        })?;
        Ok(out)
    }
    /// RFC 8032 signatures of this replica's own envelopes.
    pub fn sign(&mut self, seed: &[u8; 32], msgs: &[Envelope]) -> Result<Vec<[u8; 64]>> {
        let n = msgs.len();
        let idx = vec![0u16; n];
        let mut r = vec![[0u8; 32]; n];
        let mut s = vec![[0u8; 32]; n];
        check(unsafe {
            ffi::pbft_sign_batch(self.ctx, seed.as_ptr(), 1, idx.as_ptr(), msgs.as_ptr() as *const u8,
                                 ffi::PBFT_ENVELOPE_BYTES as u32, ffi::PBFT_ENVELOPE_BYTES as u32, n as u64,
                                 r.as_mut_ptr() as *mut u8, s.as_mut_ptr() as *mut u8, ptr::null_mut())
        })?;
        Ok(r.iter().zip(s.iter()).map(|(r, s)| {
            let mut sig = [0u8; 64];
            sig[..32].copy_from_slice(r);
            sig[32..].copy_from_slice(s);
            sig
        }).collect())
    }
    pub fn raw(&self) -> *mut ffi::pbft_ctx {
        self.ctx
    }
}

fn pack(items: &[&[u8]]) -> (Vec<u8>, Vec<u64>, Vec<u32>) {
    let mut data = Vec::new();
    let mut offs = Vec::with_capacity(items.len());
    let mut lens = Vec::with_capacity(items.len());
    for it in items {
        offs.push(data.len() as u64);
        lens.push(it.len() as u32);
        data.extend_from_slice(it);
    }
    data.extend_from_slice(&[0u8; 16]); // the digest kernels read aligned dwords past each item
    (data, offs, lens)
}

impl BatchVerifier for GpuVerifier {
    fn set_keys(&mut self, keys: &[[u8; 32]]) -> Result<Vec<bool>> {
        let mut ok = vec![0u8; keys.len()];
        check(unsafe {
            ffi::pbft_verify_set_keys(self.ctx, keys.as_ptr() as *const u8, keys.len() as u32, ok.as_mut_ptr())
        })?;
        Ok(ok.into_iter().map(|b| b == 1).collect())
    }
    fn submit(&mut self, batch: SigBatch) -> Result<Ticket> {
        if self.inflight.is_some() {
            return Err(Error { code: ffi::PBFT_EBUSY, message: "one batch in flight per context".into() });
        }
        let n = batch.len();
        let mut out = Bitmap::zeros(n);
        // pageable Vec buffers: copied into the context's pinned staging by the call, then DMA'd asynchronously
        check(unsafe {
            ffi::pbft_verify_batch_async(self.ctx, batch.r.as_ptr() as *const u8, batch.s.as_ptr() as *const u8,
                                         batch.key_idx.as_ptr(), batch.msg.as_ptr() as *const u8,
                                         ffi::PBFT_ENVELOPE_BYTES as u32, ffi::PBFT_ENVELOPE_BYTES as u32,
                                         n as u64, out.0.as_mut_ptr())
        })?;
        self.next += 1;
        self.inflight = Some((self.next, out));
        Ok(Ticket(self.next))
    }
    fn poll(&mut self, ticket: &Ticket) -> Result<Option<Bitmap>> {
        match &self.inflight {
            Some((id, _)) if *id == ticket.0 => {}
            _ => return Err(Error { code: ffi::PBFT_EINVAL, message: "unknown ticket".into() }),
        }
        match check(unsafe { ffi::pbft_verify_poll(self.ctx) }) {
            Ok(1) => Ok(Some(self.inflight.take().unwrap().1)),
            Ok(_) => Ok(None),
            Err(e) => {
                self.inflight = None; // the library dropped the failed batch
                Err(e)
            }
        }
    }
}

impl Drop for GpuVerifier {
    fn drop(&mut self) {
        unsafe {
            if self.inflight.is_some() {
                ffi::pbft_verify_wait(self.ctx);
            }
            ffi::pbft_verify_ctx_destroy(self.ctx);
        }
    }
}

/// The reference's CPU crypto path: ed25519-dalek 1.0.1 `verify_strict`, one signature at a time.
#[cfg(feature = "cpu")]
pub struct CpuVerifier {
    keys: Vec<Option<ed25519_dalek::PublicKey>>,
    done: Option<(u64, Bitmap)>,
    next: u64,
}

#[cfg(feature = "cpu")]
impl CpuVerifier {
    pub fn new() -> Self {
        CpuVerifier { keys: Vec::new(), done: None, next: 0 }
    }
}

#[cfg(feature = "cpu")]
impl BatchVerifier for CpuVerifier {
    fn set_keys(&mut self, keys: &[[u8; 32]]) -> Result<Vec<bool>> {
        // libp2p decodes the identity key once per peer (PublicKey::from_bytes = decompress);
        // verify_strict additionally rejects a small-order A at every verification
        self.keys = keys.iter().map(|k| ed25519_dalek::PublicKey::from_bytes(k).ok()).collect();
        Ok(self.keys.iter().map(|k| k.is_some()).collect())
    }
    fn submit(&mut self, batch: SigBatch) -> Result<Ticket> {
        use std::convert::TryFrom;
        let mut bm = Bitmap::zeros(batch.len());
        for i in 0..batch.len() {
            let mut sig = [0u8; 64];
            sig[..32].copy_from_slice(&batch.r[i]);
            sig[32..].copy_from_slice(&batch.s[i]);
            let ok = match (self.keys.get(batch.key_idx[i] as usize), ed25519_dalek::Signature::try_from(&sig[..])) {
                (Some(Some(pk)), Ok(sig)) => pk.verify_strict(&batch.msg[i], &sig).is_ok(),
                _ => false,
            };
            if ok {
                bm.set(i);
            }
        }
        self.next += 1;
        self.done = Some((self.next, bm));
        Ok(Ticket(self.next))
    }
    fn poll(&mut self, ticket: &Ticket) -> Result<Option<Bitmap>> {
        match self.done.take() {
            Some((id, bm)) if id == ticket.0 => Ok(Some(bm)),
            other => {
                self.done = other;
                Err(Error { code: ffi::PBFT_EINVAL, message: "unknown ticket".into() })
            }
        }
    }
}

/// libp2p PeerId (38 bytes: 00 24 08 01 12 20 || A) -> the Ed25519 key A.
pub fn key_from_peer_id(peer_id: &[u8]) -> Result<[u8; 32]> {
    let mut a = [0u8; 32];
    check(unsafe { ffi::pbft_key_from_peer_id(peer_id.as_ptr(), peer_id.len(), a.as_mut_ptr()) })?;
    Ok(a)
}

/// Round events reported by [`Replica::flush`].
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum RoundEvent {
    /// The PrePrepare's signature verified: multicast this replica's Prepare.
    PrePrepared { view: u64, seq: u64 },
    /// prepared(m, v, n): 2f matching Prepares from distinct backups: multicast the Commit.
    Prepared { view: u64, seq: u64 },
    /// committed-local: 2f+1 matching Commits: execute and reply to the client.
    CommittedLocal { view: u64, seq: u64 },
}

/// The round batcher + quorum state machine of one replica (include/pbft_replica.h).  It borrows the
/// `GpuVerifier` whose context it submits to (`'a`): the context must outlive the replica, whose Drop may
/// still wait on a batch in flight there.
pub struct Replica<'a> {
    raw: *mut ffi::pbft_replica,
    // a Rust BatchVerifier installed as the replica's asynchronous votes verifier (None: the GPU context)
    verifier: Option<Box<Backend>>,
    // event buffer reused by every flush_poll / flush (the event loop polls ~1,500 times per 2^20 round)
    events: Vec<ffi::pbft_round_event>,
    _gpu: PhantomData<&'a GpuVerifier>,
}

// A BatchVerifier behind the replica's submit / poll callbacks (pbft_replica_set_votes_verifier).
struct Backend {
    v: Box<dyn BatchVerifier>,
    pending: Option<(Ticket, *mut u64, usize)>,
}

extern "C" fn votes_submit_trampoline(user: *mut c_void, sig: *const u8, key_idx: *const u16,
                                      env_idx: *const u32, envelopes: *const u8, n_env: u32, n: u64,
                                      bitmap_out: *mut u64) -> c_int {
    let b = unsafe { &mut *(user as *mut Backend) };
    let n = n as usize;
    let mut vb = VotesBatch::default();
    unsafe {
        for row in std::slice::from_raw_parts(sig as *const [u8; 64], n) {
            let mut r = [0u8; 32];
            let mut s = [0u8; 32];
            r.copy_from_slice(&row[..32]);
            s.copy_from_slice(&row[32..]);
            vb.r.push(r);
            vb.s.push(s);
        }
        vb.key_idx.extend_from_slice(std::slice::from_raw_parts(key_idx, n));
        vb.env_idx.extend_from_slice(std::slice::from_raw_parts(env_idx, n));
        vb.envelopes.extend_from_slice(std::slice::from_raw_parts(envelopes as *const Envelope, n_env as usize));
    }
    let batch = match vb.to_sig_batch() {
        Ok(batch) => batch,
        Err(e) => return e.code,
    };
    match b.v.submit(batch) {
        Ok(t) => {
            b.pending = Some((t, bitmap_out, (n + 63) / 64));
            0
        }
        Err(e) => e.code,
    }
}

extern "C" fn votes_poll_trampoline(user: *mut c_void) -> c_int {
    let b = unsafe { &mut *(user as *mut Backend) };
    let (t, out, words) = match b.pending.take() {
        Some(p) => p,
        None => return 1,
    };
    match b.v.poll(&t) {
        Ok(Some(bm)) => {
            unsafe { ptr::copy_nonoverlapping(bm.0.as_ptr(), out, words.min(bm.0.len())) };
            1
        }
        Ok(None) => {
            b.pending = Some((t, out, words));
            0
        }
        Err(e) => e.code,
    }
}

fn round_events(ev: &[ffi::pbft_round_event]) -> Vec<RoundEvent> {
    ev.iter().filter_map(|e| match e.kind {
        ffi::PBFT_EVENT_PRE_PREPARED => Some(RoundEvent::PrePrepared { view: e.view, seq: e.seq }),
        ffi::PBFT_EVENT_PREPARED => Some(RoundEvent::Prepared { view: e.view, seq: e.seq }),
        ffi::PBFT_EVENT_COMMITTED_LOCAL => Some(RoundEvent::CommittedLocal { view: e.view, seq: e.seq }),
        _ => None,
    }).collect()
}

impl<'a> Replica<'a> {
    /// `gpu`: the context whose key set is `keys` (pbft_verify_set_keys); replica ids are
    /// positions in `keys` (network.json's "nodes" order); f = (n - 1) / 3.
    pub fn new(gpu: Option<&'a GpuVerifier>, self_id: u32, keys: &[[u8; 32]]) -> Result<Self> {
        let mut raw = ptr::null_mut();
        let ctx = gpu.map(|g| g.raw()).unwrap_or(ptr::null_mut());
        check(unsafe {
            ffi::pbft_replica_create(ctx, keys.len() as u32, self_id, keys.as_ptr() as *const u8, &mut raw)
        })?;
        Ok(Replica { raw, verifier: None, events: vec![ffi::pbft_round_event::default(); 4096], _gpu: PhantomData })
    }
    /// One replica over several GPU contexts (one per GPU of the node, each with `keys` installed;
    /// pbft_replica_create_multi): a large flush is cut into one slice per context, staged and launched
    /// on every GPU's own PCIe link at once, and applied in row order as each slice's bitmap lands.
    pub fn new_multi(gpus: &[&'a GpuVerifier], self_id: u32, keys: &[[u8; 32]]) -> Result<Self> {
        let ctxs: Vec<*mut ffi::pbft_ctx> = gpus.iter().map(|g| g.raw()).collect();
        let mut raw = ptr::null_mut();
        check(unsafe {
            ffi::pbft_replica_create_multi(ctxs.as_ptr(), ctxs.len() as u32, keys.len() as u32, self_id,
                                           keys.as_ptr() as *const u8, &mut raw)
        })?;
        Ok(Replica { raw, verifier: None, events: vec![ffi::pbft_round_event::default(); 4096], _gpu: PhantomData })
    }
    /// Back the batcher with any BatchVerifier (e.g. CpuVerifier) instead of the GPU context; its
    /// submit / poll become the replica's flush_submit / flush_poll.
    pub fn set_verifier(&mut self, v: Box<dyn BatchVerifier>) -> Result<()> {
        let mut boxed = Box::new(Backend { v, pending: None });
        let user = &mut *boxed as *mut Backend as *mut c_void;
        check(unsafe {
            ffi::pbft_replica_set_votes_verifier(self.raw, votes_submit_trampoline, votes_poll_trampoline, user)
        })?;
        self.verifier = Some(boxed);
        Ok(())
    }
    /// Peers admitted after start-up (Pbft::add_peer, src/behavior.rs:45-61): replica `idx[i]` gets `keys[i]`
    /// (its PeerId resolves through `peer_index` from now on; with a GPU context only its tables are rebuilt).
    pub fn update_keys(&mut self, idx: &[u32], keys: &[[u8; 32]]) -> Result<Vec<bool>> {
        if idx.len() != keys.len() {
            return Err(Error { code: ffi::PBFT_EINVAL, message: "update_keys: idx and keys lengths differ".into() });
        }
        let mut ok = vec![0u8; keys.len()];
        check(unsafe {
            ffi::pbft_replica_update_keys(self.raw, idx.as_ptr(), keys.as_ptr() as *const u8, keys.len() as u32,
                                          ok.as_mut_ptr())
        })?;
        Ok(ok.into_iter().map(|b| b == 1).collect())
    }
    /// PrePrepare ingress (validate_pre_prepare, src/behavior.rs:126-157, plus the signature TODO :127) from
    /// replica `peer` -- the AUTHENTICATED connection's replica index (`peer_index` of inject_node_event's
    /// peer_id, src/behavior.rs:304); dropped unless it is the view's primary.
    pub fn on_pre_prepare(&mut self, peer: u32, view: u64, seq: u64, operation: &[u8], digest: &[u8; 64],
                          primary_sig: &[u8; 64]) -> Result<bool> {
        let rc = check(unsafe {
            ffi::pbft_replica_on_pre_prepare(self.raw, peer, view, seq, operation.as_ptr(), operation.len() as u32,
                                             digest.as_ptr(), primary_sig.as_ptr(), ptr::null_mut())
        })?;
        Ok(rc == 1)
    }
    /// Many pushes at once (e.g. one decoded read of every connection); returns how many were queued.
    pub fn push_many(&mut self, kind: &[u8], view: &[u64], seq: &[u64], digests: &[[u8; 64]], signer: &[u32],
                     sigs: &[[u8; 64]]) -> Result<u64> {
        let n = kind.len();
        if view.len() != n || seq.len() != n || digests.len() != n || signer.len() != n || sigs.len() != n {
            return Err(Error { code: ffi::PBFT_EINVAL, message: "push_many: column lengths differ".into() });
        }
        let mut q = 0u64;
        check(unsafe {
            ffi::pbft_replica_push_many(self.raw, n as u64, kind.as_ptr(), view.as_ptr(), seq.as_ptr(),
                                        digests.as_ptr() as *const u8, signer.as_ptr(), sigs.as_ptr() as *const u8,
                                        &mut q)
        })?;
        Ok(q)
    }
    /// A Prepare / Commit from the AUTHENTICATED peer `signer` (inject_node_event's peer_id).
    pub fn push(&mut self, kind: u8, view: u64, seq: u64, digest: &[u8; 64], signer: u32, sig: &[u8; 64])
                -> Result<bool> {
        let rc = check(unsafe {
            ffi::pbft_replica_push(self.raw, kind, view, seq, digest.as_ptr(), signer, sig.as_ptr())
        })?;
        Ok(rc == 1)
    }
    /// Raw UviBytes/JSON frames read from peer `peer_idx`'s connection; returns bytes consumed
    /// (keep the rest for the next read).
    pub fn push_frames(&mut self, peer_idx: u32, stream: &[u8]) -> Result<usize> {
        let (mut used, mut pushed, mut dropped) = (0u64, 0u64, 0u64);
        check(unsafe {
            ffi::pbft_replica_push_frames(self.raw, peer_idx, stream.as_ptr(), stream.len(), &mut used,
                                          &mut pushed, &mut dropped)
        })?;
        Ok(used as usize)
    }
    /// 160-byte binary records (pbft_wire.h PBFT_RECORD_BYTES) read from peer `peer_idx`'s connection;
    /// returns (bytes consumed, votes pushed, records dropped) -- keep the unconsumed tail for the next read.
    pub fn push_records(&mut self, peer_idx: u32, stream: &[u8]) -> Result<(usize, u64, u64)> {
        let (mut used, mut pushed, mut dropped) = (0u64, 0u64, 0u64);
        check(unsafe {
            ffi::pbft_replica_push_records(self.raw, peer_idx, stream.as_ptr(), stream.len(), &mut used,
                                           &mut pushed, &mut dropped)
        })?;
        Ok((used as usize, pushed, dropped))
    }
    /// Where the last push_many and the last flush spent their time (host clock, ns).
    pub fn timings(&self) -> Result<ffi::pbft_replica_timings> {
        let mut t = ffi::pbft_replica_timings::default();
        check(unsafe { ffi::pbft_replica_get_timings(self.raw, &mut t) })?;
        Ok(t)
    }
    /// Launch one batch of every ready sub-window (force = the deadline: everything pending) without
    /// waiting for it; returns its signatures (0: nothing launched).  Err(PBFT_EBUSY) while one is in flight.
    pub fn flush_submit(&mut self, force: bool) -> Result<u64> {
        let mut n = 0u64;
        check(unsafe { ffi::pbft_replica_flush_submit(self.raw, force as c_int, &mut n) })?;
        Ok(n)
    }
    /// Call from NetworkBehaviour::poll (src/behavior.rs:416-426): None while the GPU works, else the round
    /// events decided by the finished batch (and any still queued).
    pub fn flush_poll(&mut self) -> Result<Option<Vec<RoundEvent>>> {
        let mut n = 0u32;
        let rc = check(unsafe {
            ffi::pbft_replica_flush_poll(self.raw, self.events.as_mut_ptr(), self.events.len() as u32, &mut n)
        })?;
        if rc == 0 {
            return Ok(None);
        }
        Ok(Some(round_events(&self.events[..n as usize])))
    }
    /// Blocking: verify every ready sub-window in one batch and report new round events.
    pub fn flush(&mut self, force: bool) -> Result<Vec<RoundEvent>> {
        let mut n = 0u32;
        check(unsafe {
            ffi::pbft_replica_flush(self.raw, force as c_int, self.events.as_mut_ptr(), self.events.len() as u32,
                                    &mut n)
        })?;
        Ok(round_events(&self.events[..n as usize]))
    }
    /// The replica index of an authenticated connection's PeerId (None: not a replica).
    pub fn peer_index(&self, peer_id: &[u8]) -> Option<u32> {
        let rc = unsafe { ffi::pbft_replica_peer_index(self.raw, peer_id.as_ptr(), peer_id.len()) };
        if rc >= 0 { Some(rc as u32) } else { None }
    }
    pub fn stable_checkpoint(&mut self, seq: u64) -> Result<()> {
        check(unsafe { ffi::pbft_replica_stable_checkpoint(self.raw, seq) }).map(|_| ())
    }
    pub fn stats(&self) -> ffi::pbft_replica_stats {
        let mut s = ffi::pbft_replica_stats::default();
        unsafe { ffi::pbft_replica_get_stats(self.raw, &mut s) };
        s
    }
}

impl Drop for Replica<'_> {
    fn drop(&mut self) {
        // destroy completes a batch in flight (through the installed verifier) before `verifier` is dropped
        unsafe { ffi::pbft_replica_destroy(self.raw) };
    }
}

/// Several GPUs of this process with the round's bitmap words all-gathered on RCCL
/// (pbft_multi_create / pbft_verify_batch_device_multi).  Borrows its `GpuVerifier`s (`'a`):
/// their contexts must outlive it (Drop synchronises their streams).
pub struct MultiGpu<'a> {
    raw: *mut ffi::pbft_multi,
    _gpus: PhantomData<&'a GpuVerifier>,
}

impl<'a> MultiGpu<'a> {
    /// One context per device, in rank order.
    pub fn new(gpus: &[&'a GpuVerifier]) -> Result<Self> {
        let ctxs: Vec<*mut ffi::pbft_ctx> = gpus.iter().map(|g| g.raw()).collect();
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::pbft_multi_create(ctxs.as_ptr(), ctxs.len() as u32, &mut raw) })?;
        Ok(MultiGpu { raw, _gpus: PhantomData })
    }
    /// Enqueue: rank r verifies its device-resident shard; every rank's `d_bitmap[r]` then holds the round
    /// (rank-major, `words_per_rank` words per rank).  # Safety: device pointers as in include/pbft_verify.h.
    pub unsafe fn verify_device(&mut self, d_r: &[*const u8], d_s: &[*const u8], d_key_idx: &[*const u16],
                                d_msg: &[*const u8], n: &[u64], words_per_rank: u64,
                                d_bitmap: &[*mut u64]) -> Result<()> {
        check(ffi::pbft_verify_batch_device_multi(self.raw, d_r.as_ptr(), d_s.as_ptr(), d_key_idx.as_ptr(),
                                                  d_msg.as_ptr(), ffi::PBFT_ENVELOPE_BYTES as u32,
                                                  ffi::PBFT_ENVELOPE_BYTES as u32, n.as_ptr(), words_per_rank,
                                                  d_bitmap.as_ptr())).map(|_| ())
    }
    pub fn sync(&mut self) -> Result<()> {
        check(unsafe { ffi::pbft_multi_sync(self.raw) }).map(|_| ())
    }
}

impl Drop for MultiGpu<'_> {
    fn drop(&mut self) {
        unsafe { ffi::pbft_multi_destroy(self.raw) };
    }
}
