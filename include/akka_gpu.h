/*
 * akka_gpu.h — C ABI of the MI355X batched actor-dispatch engine.
 *
 * This is the drop-in boundary for Akka's Dispatcher/Mailbox hot loop
 * (SURVEY.md §8(b)).  A JVM host (JNI or Panama) or the
 * Python host in akka_amd/ binds exactly these symbols.  Plain C types only:
 * no torch, no HIP types, no exceptions cross this boundary; every function
 * returns an agx_status (0 = OK).
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to /root/reference, aliases as in SURVEY.md):
 *
 *   agx_create          <- MessageDispatcherConfigurator.dispatcher() +
 *                          Dispatchers.configuratorFrom
 *                          (akka-actor/src/main/scala/akka/dispatch/AbstractDispatcher.scala:338-347,
 *                           akka-actor/src/main/scala/akka/dispatch/Dispatchers.scala:235-262)
 *                          with MailboxType.create for the bounded/unbounded queue
 *                          (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:638-640,
 *                           akka-actor/src/main/scala/akka/dispatch/Mailboxes.scala:204-260)
 *   agx_register_range  <- MessageDispatcher.attach / ActorCell.init (Create) for a
 *                          contiguous range of fixed-layout actors
 *                          (AbstractDispatcher.scala:145-148, akka-actor/.../actor/dungeon/Dispatch.scala:63-100)
 *   agx_stage_tells     <- LocalActorRef.! -> ActorCell.sendMessage -> Dispatcher.dispatch
 *                          (akka-actor/.../actor/ActorRef.scala:412-413, ActorCell.scala:325-326,
 *                           akka-actor/.../dispatch/Dispatcher.scala:61-65)
 *   agx_run             <- registerForExecution + Mailbox.run/processMailbox on the
 *                          ForkJoinPool, as BSP supersteps
 *                          (Dispatcher.scala:120-143, Mailbox.scala:227-277)
 *   agx_read_state      <- (no reference counterpart: actor state is private to the
 *                          JVM object; the GPU engine exposes it for the host/oracle)
 *   agx_set_mailbox_class / agx_set_mailbox
 *                       <- Mailboxes.lookupConfigurator / getMailboxType per actor
 *                          (akka-actor/.../dispatch/Mailboxes.scala:140-191,204-260)
 *   agx_set_outbound / agx_take_outbound
 *                       <- sender() ! reply to a JVM actor (akka-actor/.../actor/ActorCell.scala:583-587):
 *                          GPU tells to host-side actors leave the engine through an outbox
 *   agx_destroy         <- MessageDispatcher.shutdown (AbstractDispatcher.scala:325)
 *
 * Threading: an engine handle is driven by one host thread at a time (the
 * single-writer-per-actor rule at engine granularity, Mailbox.scala:185-203) -- except agx_tell,
 * which any thread may call at any time (the lock-free tell path, below).
 */
#ifndef AKKA_GPU_H
#define AKKA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AGX_ABI_VERSION 1u

typedef int32_t agx_status;
#define AGX_OK 0
#define AGX_EINVAL 1    /* bad argument / configuration                     */
#define AGX_ENOMEM 2    /* device or host allocation failed                 */
#define AGX_EDEVICE 3   /* HIP runtime error (message via agx_last_error)   */
#define AGX_ECOMM 4     /* RCCL error                                       */
#define AGX_ECAPACITY 5 /* in-flight messages exceed the engine's capacity  */
#define AGX_ESTATE 6    /* call not valid in the engine's current state     */
#define AGX_ERANGE 7    /* a GCounter / PNCounter slot passed 2^64 - 1: the reference's BigInt
                           (DD/GCounter.scala:53) has no bound, the u64 slot wrapped */

/* "no sender" (Actor.noSender / deadLetters as sender, AbstractDispatcher.scala:29-37) */
#define AGX_NO_SENDER 0xFFFFFFFFu

/* Behaviour kinds: the fixed-layout subset of typed Behaviors.receive
 * (akka-actor-typed/.../scaladsl/Behaviors.scala:101-121).  Each returns
 * same / stopped / unhandled (TY/Behavior.scala:229-278,
 * TY/internal/adapter/ActorAdapter.scala:152-168).  State words are u64.   */
enum agx_behavior_kind {
  AGX_KIND_NONE = 0,       /* unregistered: every message is a dead letter            */
  AGX_KIND_COUNTER = 1,    /* w0 += 1; w1 += payload                                  */
  AGX_KIND_RING = 2,       /* w0 += 1; payload>0 -> tell((self+stride)%N, payload-1)  */
  AGX_KIND_FANOUT = 3,     /* w0 += 1; w1 += payload; ttl=pay>>24 >0 -> k Zipf tells  */
  AGX_KIND_FORWARD_RR = 4, /* w0 += 1; payload>0 -> tell(next out-edge RR, payload-1) */
  AGX_KIND_STOP_AFTER = 5, /* w0 += 1; w0 >= w1 -> Behaviors.stopped                  */
  AGX_KIND_PINGPONG = 6,   /* BenchmarkActors.PingPong: reply to sender, stop at 0    */
  AGX_KIND_EVEN = 7,       /* odd payload -> Behaviors.unhandled; else w0 += 1         */
  /* Replicator-style CRDT replicas (akka-distributed-data), see "CRDT behaviours" below */
  AGX_KIND_GCOUNTER = 8,   /* w[0..7]  = GCounter slots                                 */
  AGX_KIND_PNCOUNTER = 9,  /* w[0..7]  = increments, w[8..15] = decrements              */
  AGX_KIND_ORSET = 10,     /* w[0..259] = 64 x 8 u32 dots + 8 u32 version vector        */
  AGX_KIND_MAX = 11
};

/* Behaviour results (ActorAdapter.next, TY/internal/adapter/ActorAdapter.scala:152-168) */
#define AGX_RES_SAME 0u
#define AGX_RES_STOPPED 1u
#define AGX_RES_UNHANDLED 2u
#define AGX_RES_BECOME 3u /* compiled behaviours: the next behaviour is agx_case.next */

/* --- compiled behaviours ------------------------------------------------------
 * A typed Behaviors.receiveMessage / javadsl ReceiveBuilder subset lowered to tables
 * (akka_amd/typed.py is the lowering; TY/scaladsl/Behaviors.scala:101-121,
 * TY/javadsl/ReceiveBuilder.scala:48-98,209-218).  An actor of kind AGX_KIND_COMPILED + b
 * runs behaviour b: cases [first[b], first[b+1]) are tried in order and the first whose
 * message tests and state guard hold runs its actions, then returns its result --
 * Behaviors.same, stopped, unhandled, or a become to behaviour `next` (stored in the
 * actor's kind byte).  No matching case = Behaviors.unhandled (ReceiveBuilder.receive).
 * Compiled behaviours keep their state in words 0 and 1 (two u64 fields).
 * Operands: value = base(src, word) + k, base = 0 (AGX_V_CONST), the payload, its tag
 * (payload >> 24), its argument (payload & 0xFFFFFF), state word `word`, the sender id or
 * the actor's own id.  Comparisons are unsigned 64-bit.                              */
#define AGX_KIND_COMPILED 16u
#define AGX_MAX_BEHAVIORS 64u
#define AGX_MAX_CASES 1024u
#define AGX_MAX_ACTS 4096u
enum agx_operand { AGX_V_CONST = 0, AGX_V_PAYLOAD = 1, AGX_V_TAG = 2, AGX_V_ARG = 3, AGX_V_WORD = 4,
                   AGX_V_SENDER = 5, AGX_V_SELF = 6 };
enum agx_cmp { AGX_CMP_ANY = 0, AGX_CMP_EQ = 1, AGX_CMP_NE = 2, AGX_CMP_LT = 3, AGX_CMP_LE = 4, AGX_CMP_GT = 5,
               AGX_CMP_GE = 6 };
enum agx_action_op {
  AGX_A_SET = 1,  /* word[w] = operand                                          */
  AGX_A_ADD = 2,  /* word[w] += operand (wrapping)                              */
  AGX_A_MAX = 3,  /* word[w] = max(word[w], operand)                            */
  AGX_A_MIN = 4,
  AGX_A_TELL = 5  /* tell(dst operand, payload): payload = (u32)operand, or with a message tag
                     (or_mask != 0) (operand & 0xFFFFFF) | or_mask; a dst operand based on the
                     actor's own id is taken mod n_actors (ring neighbours); an unknown id is a
                     dead letter */
};
typedef struct agx_case {
  uint8_t src1, word1, cmp1, src2; /* test 1: operand(src1, word1, k1) cmp1 operand(src2, word2, k2) */
  uint8_t word2, src3, word3, cmp2; /* test 2: operand(src3, word3, k3) cmp2 operand(src4, word4, k4) */
  uint8_t src4, word4, result, next;
  uint16_t act_first, act_count;    /* actions [act_first, act_first + act_count) */
  int64_t k1, k2, k3, k4;
} agx_case; /* 48 B */
typedef struct agx_act {
  uint8_t op, word, src, sword;     /* action; target word; operand (src, sword, k)  */
  uint8_t dsrc, dword, pad0, pad1;  /* AGX_A_TELL destination operand (dsrc, dword, dk) */
  uint32_t or_mask;                 /* AGX_A_TELL: payload |= or_mask (a message tag)  */
  int64_t k, dk;
} agx_act; /* 32 B */

#define AGX_MAX_WORDS 656u /* = AGX_ORSET_DELTA_WORDS (the widest layout) */
#define AGX_MAX_RANKS 16u

/* --- CRDT behaviours ---------------------------------------------------------
 * Each actor of a CRDT kind is one replica holding one data value; its node
 * index (the UniqueAddress slot, akka-cluster/.../Member.scala:307-311) is
 * id % AGX_CRDT_NODES.  Two message shapes:
 *  - control tells: payload = (op << 24) | arg, from the host or from itself
 *      AGX_OP_INCREMENT  arg = n    GCounter.increment / PNCounter.increment
 *                                   (DD/GCounter.scala:97-111, DD/PNCounter.scala:161-176)
 *      AGX_OP_DECREMENT  arg = n    PNCounter.decrement (:167-176)
 *      AGX_OP_ADD        arg = e    ORSet.add (DD/ORSet.scala:339-351), e < 64
 *      AGX_OP_REMOVE     arg = e    ORSet.remove (:380-387)
 *      AGX_OP_CLEAR                 ORSet.clear (:404-412)
 *      AGX_OP_GOSSIP     arg = k    Replicator GossipTick (DD/Replicator.scala:1316,2029-2061):
 *                                   send the full state to `fanout` random peers
 *                                   and, if k > 0, GOSSIP(k-1) to itself
 *  - state gossip: a full-state snapshot; the receiver merges it
 *    (GCounter.merge :113-125, PNCounter.merge :178, ORSet.merge :427-452).
 *    On the wire the sender field carries AGX_WIDE_BIT and the payload is
 *    (data type << 30) | an engine-internal handle to the snapshot (type =
 *    kind - AGX_KIND_GCOUNTER).  A gossip of another data type, and any state
 *    gossip reaching a non-CRDT behaviour, is Behaviors.unhandled.  Host
 *    tells are always control tells.
 * Unknown ops are Behaviors.unhandled.                                       */
#define AGX_CRDT_NODES 8u
#define AGX_ORSET_ELEMS 64u
#define AGX_GCOUNTER_WORDS 8u
#define AGX_PNCOUNTER_WORDS 16u
#define AGX_ORSET_WORDS 260u /* (64 * 8 + 8) u32 */
#define AGX_WIDE_BIT 0x80000000u
#define AGX_OP_INCREMENT 1u
#define AGX_OP_DECREMENT 2u
#define AGX_OP_ADD 3u
#define AGX_OP_REMOVE 4u
#define AGX_OP_CLEAR 5u
#define AGX_OP_GOSSIP 6u
#define AGX_OP_DELTA_TICK 7u
#define AGX_OP(op, arg) (((uint32_t)(op) << 24) | ((uint32_t)(arg) & 0xFFFFFFu))

/* --- delta-CRDT replication (agx_set_delta_crdt; Replicator delta-crdt.enabled) --------
 * Replicas form keys of AGX_CRDT_NODES consecutive ids (key = id / 8, node = id % 8): the
 * 8 replicas of a key are the key's DataEnvelopes on 8 Replicator nodes, and gossip (full
 * state and deltas) only flows between them.  Each replica's state words are the data
 * words followed by the envelope/selector area and a delta log (u32 view, D = data words):
 *   u32[2D + 0..7]    DataEnvelope.deltaVersions (seqNr last applied per node; DD/Replicator.scala:910-917)
 *   u32[2D + 8]       DeltaPropagationSelector.deltaCounter  (DD/DeltaPropagationSelector.scala:44-57)
 *   u32[2D + 9]       deltaNodeRoundRobinCounter
 *   u32[2D + 10..17]  deltaSentToNode per node (0 = nothing sent)
 *   deltaEntries --
 *     counters, u32[2D + 24 ..+ AGX_COUNTER_DELTA_U32]: {seqNr, value lo, hi} of the last increments
 *       delta, the same of the last decrements delta, the last NoDeltaPlaceholder's seqNr, 0.  A
 *       counter delta is the updated slot's new value and the own slots never decrease, so the
 *       slot-max merge of the deltas after any seqNr j is these last deltas (or a placeholder if
 *       one lies after j): unbounded, as the reference's map (DD/DeltaPropagationSelector.scala:149-155).
 *     ORSet, u32[2D + 24 + AGX_DELTA_LOG_U32(1) * (seq % AGX_DELTA_LOG) ...], a ring:
 *       {seq, type (1 AddDeltaOp, 2 RemoveDeltaOp, 3 FullStateDeltaOp) | elem << 8, version, 0, vvector[8]};
 *       an ORSet replica that would overwrite a seqNr some node has not been sent reports
 *       AGX_ECAPACITY (the one bounded difference from the reference).
 * Ops on a delta replica:
 *   AGX_OP_DELTA_TICK  arg = k | AGX_DELTA_WRITE?   DeltaPropagationTick (DD/Replicator.scala:1953-1963):
 *       (AGX_DELTA_WRITE: first tell itself one seeded local update -- a writer client), then for
 *       each node of this tick's round-robin slice with deltas after deltaSentToNode, merge them
 *       into one delta group (DeltaOp.merge, max-delta-size) and tell that replica a
 *       DeltaPropagation(fromSeqNr, toSeqNr); if k > 0, DELTA_TICK(k-1) to itself.
 *   a DeltaPropagation is applied with causal delivery for ORSet (skip if already handled or a
 *   seqNr is missing, DD/Replicator.scala:1965-2027) and ORSet.mergeDelta (DD/ORSet.scala:455-501);
 *   counters merge it (no causal delivery needed).  A group that is a NoDeltaPlaceholder
 *   (too large, or a no-op update in range) is not told (createDeltaPropagation leaves it out,
 *   DD/Replicator.scala:1364,1957); deltaSentToNode still advances.                           */
#define AGX_DELTA_WRITE 0x800000u
#define AGX_DELTA_LOG 64u            /* ORSet ring entries per replica (seqNrs not yet sent to every node) */
#define AGX_COUNTER_DELTA_U32 8u     /* counters: the last delta per slot + the last placeholder      */
#define AGX_DELTA_ENV_WORDS 12u      /* u64 words of the envelope / selector area */
#define AGX_DELTA_MAX_SIZE 50u       /* Replicator max-delta-size (reference.conf delta-crdt) */
#define AGX_DELTA_LOG_U32(orset) ((orset) ? 12u : 4u)
/* CRDT message rows (u32).  Full state: the data words, then (delta mode) deltaVersions[8].
 * DeltaPropagation (payload carries AGX_DELTA_ROW_BIT):
 *   [0] ops in the group (bit 31: NoDeltaPlaceholder) [1] from node [2] fromSeqNr [3] toSeqNr
 *   [4..11] the sender's deltaVersions, then the body --
 *   counters: [12] 1 = increments slot present | 2 = decrements slot present, [13..14] / [15..16] values;
 *   ORSet, per op: [type | n << 8] then AddDeltaOp: vvector(from), n x (element, version);
 *     RemoveDeltaOp: element, deltaDot version, vvector[8];  FullStateDeltaOp: vvector[8].
 * A group has < max-delta-size (<= 50) ops over <= AGX_DELTA_LOG seqNrs: <= 574 u32.  The row's
 * last word (pitch - 1) holds its used length in u32 (a queued row is copied forward that far). */
#define AGX_DELTA_ROW_BIT 0x20000000u
#define AGX_ORSET_DELTA_ROW_U32 576u
#define AGX_GCOUNTER_DELTA_WORDS (AGX_GCOUNTER_WORDS + AGX_DELTA_ENV_WORDS + AGX_COUNTER_DELTA_U32 / 2u)
#define AGX_PNCOUNTER_DELTA_WORDS (AGX_PNCOUNTER_WORDS + AGX_DELTA_ENV_WORDS + AGX_COUNTER_DELTA_U32 / 2u)
#define AGX_ORSET_DELTA_WORDS (AGX_ORSET_WORDS + AGX_DELTA_ENV_WORDS + AGX_DELTA_LOG * 6u)

typedef struct agx_cfg {
  uint32_t abi_version;   /* must be AGX_ABI_VERSION                                   */
  uint32_t device;        /* HIP device ordinal                                        */
  uint64_t n_actors;      /* global actor population (ids 0..n_actors-1), < 2^31       */
  uint32_t throughput;    /* dispatcher `throughput` (RC:541); <=0 behaves as 1 (Mailbox.scala:261) */
  uint32_t capacity;      /* bounded mailbox capacity C (Mailboxes.scala:212-216); 0 = unbounded */
  uint32_t n_words;       /* u64 state words per actor, 1..AGX_MAX_WORDS               */
  uint32_t max_emit;      /* max tells one message may emit (kmax)                     */
  uint32_t n_ranks;       /* GPUs the population is hash-sharded over (1 = single GPU) */
  uint32_t rank;          /* this engine's rank                                        */
  uint32_t num_shards;    /* ShardRegion number-of-shards (1000 in typed sharding)     */
  uint32_t bucket_actors;  /* actors per apply bucket: 0 = 2048, else a power of two in [32, 2048].
                             One workgroup drains a bucket; a bucket whose inbox exceeds 2048
                             messages takes the skew path -- populations with deep mailboxes
                             (ping-pong pairs, CRDT replicas with gossips) want small buckets */
  uint64_t msg_capacity;  /* max messages in flight on this rank (0 = 4 x local actors)*/
} agx_cfg;

typedef struct agx_stats {
  uint64_t delivered;     /* ActorCell.invoke calls (ActorCell.scala:539)              */
  uint64_t dead_letters;  /* overflow + to-stopped + to-unknown (Mailbox.scala:337-351,422-428) */
  uint64_t unhandled;     /* Behaviors.unhandled results (subset of delivered)         */
  uint64_t emitted;       /* tells emitted by behaviours                               */
  uint64_t staged;        /* tells staged from the host                                */
  uint64_t supersteps;    /* supersteps that had messages                              */
  uint64_t in_flight;     /* backlog + undelivered tells left when agx_run returned    */
  uint64_t bytes_alg;     /* algorithmic HBM bytes (SURVEY.md §8(d) formula)           */
} agx_stats;

typedef struct agx_engine agx_engine;

/* --- lifecycle ------------------------------------------------------------ */
agx_status agx_create(const agx_cfg* cfg, agx_engine** out);
agx_status agx_destroy(agx_engine* eng);
const char* agx_last_error(void);
uint32_t agx_abi_version(void);
/* 16 hex digits: the hash of the sources this library was built from (a build check, no
 * reference counterpart; __graft_entry__.source_hash computes the same over csrc/ and this header) */
const char* agx_build_hash(void);

/* --- actor registration (actorOf for a contiguous id range) --------------- */
/* init_state: count x state_stride bytes, actor-major, n_words u64 used per actor
 * (may be NULL = zero state).  Only ids owned by this rank are kept.         */
agx_status agx_register_range(agx_engine* eng, uint64_t first_id, uint64_t count,
                              uint32_t kind, const void* init_state, size_t state_stride);

/* --- behaviour parameters --------------------------------------------------- */
agx_status agx_set_ring(agx_engine* eng, uint32_t stride);
/* Zipf targets: cdf[i] = ceil(2^32 * P(rank <= i)) - 1 style u32 thresholds
 * (non-decreasing, cdf[n-1] = 0xFFFFFFFF); perm maps rank -> actor id.      */
agx_status agx_set_fanout(agx_engine* eng, uint32_t k, uint64_t seed, const uint32_t* cdf,
                          const uint32_t* perm, uint64_t n);
/* CRDT gossip: each GOSSIP tick sends the replica's state to `fanout` peers
 * drawn uniformly from the other actors with the counter RNG (seed, self,
 * countdown, j) — Replicator.selectRandomNode (DD/Replicator.scala:2063-2064). */
agx_status agx_set_gossip(agx_engine* eng, uint32_t fanout, uint64_t seed);
/* Delta-CRDT replication (Replicator `delta-crdt.enabled = on`, `max-delta-size`,
 * akka-distributed-data/src/main/resources/reference.conf:65-72): 0 = off (full-state
 * gossip among all replicas of one key), 1..AGX_DELTA_MAX_SIZE = on, with keys of 8 replicas
 * (see "delta-CRDT replication" above).  Call before the first agx_run; CRDT actors then need
 * n_words >= the *_DELTA_WORDS of their kind.                                               */
agx_status agx_set_delta_crdt(agx_engine* eng, uint32_t max_delta_size);
/* Compiled behaviours (see "compiled behaviours" above): behaviour b = cases
 * [first[b], first[b+1]); first has n_behaviors + 1 entries.  Replaces the tables of an
 * earlier call; call before agx_run.  Register actors with kind AGX_KIND_COMPILED + b.      */
agx_status agx_set_behaviors(agx_engine* eng, const agx_case* cases, uint32_t n_cases, const agx_act* acts,
                             uint32_t n_acts, const uint32_t* first, uint32_t n_behaviors);
/* Out-edge lists in CSR over GLOBAL ids: row_ptr[n_actors+1], col[row_ptr[n]].  */
agx_status agx_set_graph(agx_engine* eng, const uint64_t* row_ptr, const uint32_t* col);
/* The same CSR with the destinations generated on the device (workload setup for
 * 10^8-actor graphs; not part of the dispatcher boundary): edge e gets the R-MAT
 * destination of `bits` quadrant draws q = splitmix64(e*64 + bit + seed) & 0xFFFF,
 * destination bit = (ta <= q < tb) | (q >= tc), reduced mod n_actors.          */
agx_status agx_set_graph_rmat(agx_engine* eng, const uint64_t* row_ptr, uint32_t bits, uint32_t ta,
                              uint32_t tb, uint32_t tc, uint64_t seed);

/* --- tell / run ------------------------------------------------------------- */
/* Host tells (caller-owned buffers, copied).  src may be AGX_NO_SENDER.
 * Tells whose dst is not owned by this rank are ignored on this rank.
 * All or nothing: AGX_EINVAL (a tagged sender) or AGX_ECAPACITY (the tells would take the
 * messages in flight on this rank past msg_capacity) stages none of them and leaves every
 * counter unchanged -- run the engine to drain it and stage again.                              */
agx_status agx_stage_tells(agx_engine* eng, const uint32_t* dst, const uint32_t* src,
                           const uint32_t* payload, size_t n);
/* The lock-free tell path (ActorRef.! from any thread; the reference: one getAndSet enqueue,
 * akka-actor/src/main/java/akka/dispatch/AbstractNodeQueue.java:79-82, and a CAS-guarded schedule,
 * akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:185-194 + Dispatcher.scala:120-128).
 * agx_tell may be called from any number of threads at once, also while one thread is inside
 * agx_run: each calling thread appends to a queue of its own (wait-free, each sender's tells in
 * order; the next agx_run takes them as agx_stage_tells would).  *schedule = 1 iff this tell moved
 * the engine from idle to scheduled: the caller then submits ONE pump task (a task that calls
 * agx_run and then agx_pump_idle); N tells to an idle engine submit one.  agx_pump_idle is the
 * pump's last call (Mailbox.run's finally: setAsIdle, then registerForExecution if the mailbox
 * still has messages, Mailbox.scala:227-240): *reschedule = 1 iff tells arrived after the pump's
 * last agx_run, or tells are still queued because they did not fit the message capacity, or the
 * last agx_run succeeded and left mail in flight (a superstep budget) -- submit the pump again.
 * Tells are never refused or lost at capacity: agx_run takes only as many queued tells as fit
 * msg_capacity beside the mail already in flight, the rest wait in the queue for a later pump
 * (back-pressure, as an unbounded MPSC mailbox never refuses an enqueue, AbstractNodeQueue.java:
 * 79-82; a bounded mailbox class still tail-drops at its own capacity).  agx_pump_cancel: the pump
 * could not be submitted (the executor rejected it): the engine goes back to idle without the
 * re-check, so the next tell schedules it again (Dispatcher.registerForExecution's catch,
 * Dispatcher.scala:130-138).  (src may be AGX_NO_SENDER; schedule / reschedule may be NULL.)  */
agx_status agx_tell(agx_engine* eng, uint32_t dst, uint32_t src, uint32_t payload, int32_t* schedule);
agx_status agx_pump_idle(agx_engine* eng, int32_t* reschedule);
agx_status agx_pump_cancel(agx_engine* eng);
/* Run up to max_supersteps supersteps or until quiescent; stats are cumulative
 * over the engine's lifetime.  out may be NULL: the counters are then not read
 * back (agx_get_stats does it later, and reports AGX_ECAPACITY if an overflow
 * was recorded meanwhile).                                                    */
agx_status agx_run(agx_engine* eng, uint32_t max_supersteps, agx_stats* out);
agx_status agx_get_stats(agx_engine* eng, agx_stats* out);
/* agx_run, plus the run's device time in ms: HIP events on the engine's stream before the first
 * launch and after the last superstep (bench.py's roofline timing of graph-replayed supersteps). */
agx_status agx_run_timed(agx_engine* eng, uint32_t max_supersteps, agx_stats* out, float* device_ms);
/* Supersteps of a single-rank multi-pass engine (> 2^20 actors) whose mail needed no radix pass:
 * the previous apply's tells were already in destination order (a ring, a stencil -- identity
 * grouping).  Diagnostic; the grouping is the same either way.                  */
agx_status agx_identity_supersteps(agx_engine* eng, uint64_t* out);
/* Bounded-mailbox ring slots handed out so far (high-water mark; single-rank multi-pass engine whose
 * mailbox classes are all bounded): a bucket that holds more than one LDS tile of
 * mail keeps its actors' queued messages in per-actor rings of the largest capacity -- a queued
 * message is written once and read once -- until its rings are empty and its mail fits one tile
 * again (the slot is then reused).  Diagnostic; the semantics are the same either way. */
agx_status agx_ring_buckets(agx_engine* eng, uint64_t* out);
/* Multi-rank exchange accounting of this rank (diagnostic): out[0] supersteps on the device-resident
 * exchange (fixed per-peer slabs), out[1] supersteps on the host-planned exchange (exact per-peer
 * sizes), out[2] envelope bytes and out[3] CRDT row bytes sent to peers, out[4] 1 once the CRDT row
 * slabs did not fit on some rank (row handle space, AGX_MR_ROW_MB or memory) and every rank moved to
 * the host-planned exchange, out[5] the slab (envelopes per peer per superstep). */
agx_status agx_exchange_info(agx_engine* eng, uint64_t out[6]);
/* Persistent fused supersteps (diagnostic): out[0] replays launched as ONE persistent
 * launch (a strict replay whose supersteps are the dense launch alone: k_dense_fused runs them with a
 * grid barrier between supersteps; opt-in: AGX_PERSIST=1), out[1] supersteps they ran. */
agx_status agx_persist_info(agx_engine* eng, uint64_t out[2]);

/* --- per-actor mailboxes (Mailboxes.lookupConfigurator, Mailboxes.scala:204-260) -------------
 * An actor's mailbox type is resolved per actor in the reference (props, then dispatcher, then
 * requirement; ActorMailboxSpec.scala:245-450).  Here a dispatcher's actors use one of
 * AGX_MAX_MAILBOX_CLASSES mailbox classes: class 0 is agx_cfg.capacity, classes 1..7 are set by
 * agx_set_mailbox_class (bounded-capacity:N -> N; an unbounded mailbox type -> 0), and
 * agx_set_mailbox binds a range of actors to a class (default: class 0).  A bounded class drains at
 * most min(throughput, capacity) messages per mailbox run, as a bounded queue never holds more.    */
#define AGX_MAX_MAILBOX_CLASSES 8u
agx_status agx_set_mailbox_class(agx_engine* eng, uint32_t mailbox_class, uint32_t capacity);
agx_status agx_set_mailbox(agx_engine* eng, uint64_t first_id, uint64_t count, uint32_t mailbox_class);

/* --- the reply path: actors that live on the host ------------------------------------------
 * Ids [first_host_id, first_host_id + n_host) -- outside the population (>= n_actors, < 2^31) --
 * name host-side actors, e.g. the JVM ActorRefs that told GPU actors (their sender() ids).  A GPU
 * behaviour's tell to one of them is not a dead letter: it is appended to the engine's outbox
 * (each sender's tells in emission order; different senders interleave arbitrarily, as on the
 * JVM) and the host takes it with agx_take_outbound and delivers it.  Outbound tells leave the
 * engine: they are not counted in agx_stats.emitted.  More than `capacity` outbound tells between
 * two agx_take_outbound calls is AGX_ECAPACITY.  agx_take_outbound copies up to `cap` envelopes
 * (dst host id, src GPU actor id, payload) and removes them; *n = how many.                   */
agx_status agx_set_outbound(agx_engine* eng, uint32_t first_host_id, uint32_t n_host, uint64_t capacity);
agx_status agx_take_outbound(agx_engine* eng, uint32_t* dst, uint32_t* src, uint32_t* payload, uint64_t cap,
                             uint64_t* n);

/* --- state readback ----------------------------------------------------------- */
/* The population (agx_cfg.n_actors, all ranks) and state words per actor: the sizes a binding
 * checks caller arrays against before agx_set_graph / agx_read_state (whose pointers carry none). */
agx_status agx_get_shape(agx_engine* eng, uint64_t* n_actors, uint32_t* n_words);
/* words: count x n_words u64 (actor-major); alive: count bytes (may be NULL).
 * Only ids owned by this rank are written; others are left untouched.       */
agx_status agx_read_state(agx_engine* eng, uint64_t first_id, uint64_t count, uint64_t* words,
                          uint8_t* alive);

/* --- multi-GPU (one process per GPU, RCCL over xGMI) ------------------------- */
/* 128-byte RCCL unique id: rank 0 creates it, the host broadcasts it.        */
agx_status agx_comm_unique_id(uint8_t out[128]);
agx_status agx_comm_init(agx_engine* eng, const uint8_t id[128]);
/* Single-process loopback transport: run `n` engines (ranks 0..n-1 of one
 * population) that share one device, exchanging mail with device copies.
 * Same kernels as the RCCL path; used to test sharding on a 1-GPU box.      */
agx_status agx_group_run(agx_engine** engs, uint32_t n, uint32_t max_supersteps, agx_stats* out);

/* The device-resident replays' per-superstep decision (pure host function, no GPU; the device runs
 * the same code in k_mr_pack / k_mr_unpack, agx_kernels.h mr_decide).  `mat` as below; `slab` =
 * envelopes per fixed-size peer slab; `cap` = this rank's message capacity.  *code: 0 = exchange
 * the slabs, 1 = some sender -> receiver count (off the diagonal) exceeds the slab (the host redoes
 * this superstep's exchange exactly and grows the slabs), 2 = nothing in flight on any rank, 3 =
 * backlog + received mail would exceed `cap`.  send_off / recv_off: R + 1 entries (exclusive
 * prefixes of this rank's send counts and of its receive counts in sender-rank order; [R] = the
 * total); *n_backlog = this rank's backlog (received mail is placed after it).
 * Replaces: ShardRegion delivery to remote regions (akka-cluster-sharding/.../ShardRegion.scala:
 * 154-158 routing), batched once per superstep. */
agx_status agx_mr_plan(const uint64_t* mat, uint32_t n_ranks, uint32_t rank, uint32_t slab, uint64_t cap,
                       uint32_t* code, uint64_t* send_off, uint64_t* recv_off, uint64_t* n_backlog);

/* Exchange plan of one superstep (pure host function, no GPU).  `mat` is the
 * gathered R x (R+2) matrix, row r = rank r's [tells to rank 0..R-1,
 * n_backlog, n_staged].  Outputs (R entries each): this rank's send
 * counts/offsets into its owner-partitioned tell buffer and receive
 * counts/offsets into its sort input, where received mail follows the local
 * backlog in sender-rank order (the sharded canonical order).  *inflight =
 * global messages in flight (0 = quiescent on every rank).                  */
agx_status agx_exchange_plan(const uint64_t* mat, uint32_t n_ranks, uint32_t rank, uint64_t* send_cnt,
                             uint64_t* send_off, uint64_t* recv_cnt, uint64_t* recv_off, uint64_t* inflight);

/* --- measurement ----------------------------------------------------------- */
/* Per-kernel HIP-event timing on the engine's stream (off by default).      */
agx_status agx_profile_enable(agx_engine* eng, int on);
/* Fills up to `cap` entries; returns the number of kernel classes in *n.
 * items[k]: for "bucket_apply_dense", the profiled dense launches that took
 * every bucket (read from the device's dense_left flags after each launch:
 * the wave / block launches of those supersteps returned at entry); 0 else. */
agx_status agx_profile_read(agx_engine* eng, char (*names)[32], double* total_ms,
                            uint64_t* launches, uint64_t* items, uint32_t cap, uint32_t* n);
agx_status agx_profile_reset(agx_engine* eng);

/* --- sharding helpers (ShardRegion.HashCodeMessageExtractor) ---------------- */
/* (math.abs(entityId.hashCode) % maxNumberOfShards) with entityId = decimal id
 * (akka-cluster-sharding/.../ShardRegion.scala:154-158).  May be negative.  */
int32_t agx_shard_id(uint32_t id, uint32_t num_shards);
/* rank owning `id` = floor-mod(shard_id, n_ranks).                           */
uint32_t agx_owner(uint32_t id, uint32_t num_shards, uint32_t n_ranks);

#ifdef __cplusplus
}
#endif
#endif /* AKKA_GPU_H */
