/*
 * spai.h — C ABI of the MI355X-native batched self-play MCTS engine.
 *
 * This is the drop-in boundary for the reference's hot path
 * (joshua16266261/self-play-ai).  The reference is in-process Rust with no FFI;
 * each entry point below replaces one trait method or function of that path,
 * cited as path:line relative to the reference root.  A Rust binding that
 * implements the reference traits on top of these symbols is in INTEGRATION.md.
 *
 * Conventions
 *  - Every function returns SPAI_OK (0) or a negative spai_error.  The message
 *    of the last failure on the calling thread is spai_last_error().  The
 *    reference reports rules errors as Result<_, String> (game/mod.rs:26,31)
 *    and panics on everything else (unwrap); those panics map to error codes.
 *  - Handles are opaque.  Buffers passed in or out are caller-owned HOST
 *    memory unless a parameter says "device".  Device memory and HIP streams
 *    are owned by the engine.
 *  - No global mutable state: one engine per host thread is fully independent,
 *    mirroring one Mcts + Model per self-play worker (main.rs:169-186).  An
 *    engine handle must not be used from two threads at once.
 *  - Connect4 states cross the boundary as spai_c4_state bitboards:
 *    bit (col*7 + row) of `x` / `o` holds X's / O's stone, row 0 = bottom
 *    (connect_four.rs:18), bit 6 of every column is always clear.  X moves
 *    first; the player to move is X iff num_actions_played is even
 *    (connect_four.rs:20-26,197).
 */
#ifndef SPAI_H
#define SPAI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPAI_VERSION_MAJOR 0
#define SPAI_VERSION_MINOR 2

typedef enum spai_error {
    SPAI_OK = 0,
    SPAI_ERR_INVALID = -1,       /* bad argument / handle / shape (e.g. mask_invalid_actions length) */
    SPAI_ERR_ILLEGAL_MOVE = -2,  /* Err("Illegal move: column already filled"), connect_four.rs:193 */
    SPAI_ERR_GAME_OVER = -3,     /* Err("Game has already ended"), connect_four.rs:209 */
    SPAI_ERR_DEVICE = -4,        /* HIP runtime failure */
    SPAI_ERR_NAN = -5,           /* NaN UCB or all-zero visits: the reference panics (mcts.rs:106-109) */
    SPAI_ERR_CAPACITY = -6,      /* node arena / batch capacity exceeded */
    SPAI_ERR_UNSUPPORTED = -7    /* game or net shape not built for this device path */
} spai_error;

typedef enum spai_game { SPAI_GAME_TICTACTOE = 0, SPAI_GAME_CONNECT4 = 1, SPAI_GAME_CHESS = 2 } spai_game;
typedef enum spai_status { SPAI_ONGOING = 0, SPAI_TIED = 1, SPAI_WON = 2 } spai_status; /* game/mod.rs:9-15 */

/* Evaluator used by search.  NET is Model::predict (model/mod.rs:36-98).  UNIFORM
 * and HASH are deterministic stub evaluators (not in the reference) used to pin
 * search and self-play bit-exactly against the CPU oracle. */
typedef enum spai_eval { SPAI_EVAL_NET = 0, SPAI_EVAL_UNIFORM = 1, SPAI_EVAL_HASH = 2 } spai_eval;

/* Arithmetic of a device net.  BF16: bf16 weights and activations on the MFMA
 * matrix cores, fp32 accumulate (the throughput path).  F32: the reference's
 * own fp32 arithmetic (model/mod.rs:36-98 runs libtorch in fp32), each output
 * summed in the CPU oracle's order, for parity work. */
typedef enum spai_dtype { SPAI_DTYPE_BF16 = 0, SPAI_DTYPE_F32 = 1 } spai_dtype;

typedef struct spai_c4_state {
    uint64_t x;                  /* X stones, bit col*7+row */
    uint64_t o;                  /* O stones */
    uint8_t num_actions_played;  /* connect_four.rs:24 */
    uint8_t status;              /* spai_status, connect_four.rs:25 */
    uint8_t pad[6];
} spai_c4_state;

/* mcts::Args (mcts.rs:9-18,46-59) + SelfPlayArgs (learner_concurrent.rs:21-26,50-59),
 * reduced to what the hot path reads, plus device sizing. */
typedef struct spai_config {
    float c;                 /* PUCT constant; the reference always uses Args::default().c = 2.0 (quirk Q6) */
    uint32_t num_searches;   /* simulations per move (Args.num_searches) */
    float temperature;       /* move sampling exponent on visit counts (learner_concurrent.rs:189-190) */
    uint32_t max_trees;      /* trees (parallel games) held on the device */
    uint32_t max_moves;      /* longest game; sizes the node arena (C4: 42) */
    uint32_t eval;           /* spai_eval */
    uint64_t seed;           /* move-sampling stream: Philox(seed, game id, move number) */
} spai_config;

typedef struct spai_engine spai_engine;
typedef struct spai_net spai_net;

/* ------------------------------------------------------------------ general */
const char *spai_last_error(void);
const char *spai_version(void);
int spai_device_count(int *count);
int spai_config_default(int game, spai_config *cfg);
int spai_engine_create(int game, const spai_config *cfg, int device, spai_engine **out);
int spai_engine_destroy(spai_engine *eng);
int spai_engine_sync(spai_engine *eng);

/* ------------------------------------------------------------------ rules
 * The State trait (game/mod.rs:21-33) batched over n engine-held game slots
 * [first, first+n) laid out as struct-of-arrays bitboards in HBM. */
int spai_games_resize(spai_engine *eng, uint32_t n);                       /* n slots = State::default() */
int spai_games_reset(spai_engine *eng, uint32_t first, uint32_t n);
int spai_games_write(spai_engine *eng, uint32_t first, uint32_t n, const spai_c4_state *states);
int spai_games_read(spai_engine *eng, uint32_t first, uint32_t n, spai_c4_state *states);
/* get_valid_actions (connect_four.rs:213-225) as a bitmask: bit a = action a legal */
int spai_legal_mask(spai_engine *eng, uint32_t first, uint32_t n, uint32_t *mask);
/* get_next_state (connect_four.rs:190-211) in place; rc[i] = 0 or a spai_error for slot i
 * (slot left unchanged on error).  Returns SPAI_OK if every slot succeeded, else the first error. */
int spai_apply(spai_engine *eng, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc);
/* get_value_and_terminated (connect_four.rs:231-240) */
int spai_value_terminated(spai_engine *eng, uint32_t first, uint32_t n, float *value, uint8_t *terminated);
/* get_encoding (connect_four.rs:242-259): out [n][3][6][7] f32 */
int spai_encode(spai_engine *eng, uint32_t first, uint32_t n, float *out);
/* mask_invalid_actions (connect_four.rs:261-279): policy [n][len] -> out [n][7]; len must be 7 */
int spai_mask_invalid(spai_engine *eng, uint32_t first, uint32_t n, const float *policy, uint32_t len,
                      float *out);
/* Device-resident timing of the rules kernels on n random reachable positions:
 * ms[0] legal mask, ms[1] apply+terminal, ms[2] encode (bf16), per launch. */
int spai_rules_bench(spai_engine *eng, uint32_t n, uint32_t iters, double *ms);

/* ------------------------------------------------------------------ net
 * Net trait (model/mod.rs:22-28) + Model::predict (model/mod.rs:36-98).
 * `params` are fp32 in module construction order (torso, policy head, value
 * head; conv = weight[co][ci][3][3], bias; batch_norm = weight, bias,
 * running_mean, running_var; linear = weight[out][in], bias) — the order tch
 * registers them for model/connect_four.rs:34-44.  Device path: hidden = 64. */
int spai_net_num_params(int game, int blocks, int hidden, size_t *count);
int spai_net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params);
/* Net::new (model/mod.rs:22-28) with its weights: dtype = spai_dtype */
int spai_net_create(spai_engine *eng, int blocks, int hidden, const float *params, size_t nparams, int dtype,
                    spai_net **out);
int spai_net_destroy(spai_net *net);
/* Net::forward(x, train=false): x [n][3][6][7] f32 -> logits [n][7], value [n] (tanh) */
int spai_net_forward(spai_net *net, uint32_t n, const float *x, float *logits, float *value);
/* Model::predict: states -> masked softmax priors [n][7] (softmax then mask_invalid_actions), values [n] */
int spai_predict(spai_net *net, uint32_t n, const spai_c4_state *states, float *priors, float *values);
/* Evaluator that search uses when cfg.eval == SPAI_EVAL_NET (Mcts.model, mcts.rs:41-44) */
int spai_engine_set_net(spai_engine *eng, spai_net *net);

/* ------------------------------------------------------------------ policy
 * Policy trait methods (game/mod.rs:35-44) on a flat policy array (Connect4 7,
 * TicTacToe 9, chess 4672 = get_flat_ndarray order).  Host functions.  For
 * chess, map the index to a move with spai_chess_index_move (get_action). */
/* Policy::normalize (connect_four.rs:96-98, chess.rs:518-520): p /= ndarray sum(p) */
int spai_policy_normalize(float *p, uint32_t n);
/* Policy::get_best_action (connect_four.rs:116-124, chess.rs:535-545): index of
 * the LAST maximum under f32::total_cmp (NaN above +inf, -0 below +0) */
int spai_policy_best_action(const float *p, uint32_t n, uint32_t *index);
/* Policy::sample (connect_four.rs:104-114, chess.rs:526-533): WeightedIndex
 * (rand 0.8) over p^temperature with f32 running totals.  u01 in [0, 1) is the
 * uniform that rand's UniformFloat<f32> draws, ((u32 >> 9) as f32) * 2^-23, so a
 * caller feeding its own rng's u32 reproduces rand's choice exactly.
 * SPAI_ERR_INVALID for an empty policy, a negative/NaN weight or all-zero weights. */
int spai_policy_sample(const float *p, uint32_t n, float temperature, float u01, uint32_t *index);

/* ------------------------------------------------------------------ search
 * Tree (mcts.rs:32-39,67-89,161-192) + Mcts::search (mcts.rs:196-332).
 * Trees live in HBM; node ids are per-tree handles (stable across
 * use_subtree; they are NOT the reference's BFS re-indexed arena offsets). */
int spai_trees_create(spai_engine *eng, uint32_t n);                                   /* n x Tree::default() */
int spai_tree_reset(spai_engine *eng, uint32_t tree, const spai_c4_state *root);       /* with_root_state; NULL = default */
/* Runs num_searches iterations over trees tree_idx[0..n).  Per tree i (A = 7):
 *   policy[i*A + a]       normalized root visit counts (Policy::normalize)
 *   child_ids[i*A + k]    node id of the k-th root child (legal-action order)
 *   child_visits[i*A + k] its visit count as f32
 *   n_children[i]
 * Any output pointer may be NULL. */
int spai_search(spai_engine *eng, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                uint32_t *child_ids, float *child_visits, uint32_t *n_children);
/* Tree::use_subtree(child) for a child of the root; the new root keeps N and W (quirk Q4) */
int spai_tree_use_subtree(spai_engine *eng, uint32_t tree, uint32_t child_id);
/* arena[node].state for the root or a root child; visits / value_sum of that node (may be NULL) */
int spai_tree_node(spai_engine *eng, uint32_t tree, uint32_t node_id, spai_c4_state *state, uint32_t *visits,
                   float *value_sum);
int spai_tree_size(spai_engine *eng, uint32_t tree, uint32_t *nodes);

/* ------------------------------------------------------------------ self-play
 * SelfPlayWorker::self_play (learner_concurrent.rs:169-242): n_games trees
 * from the default state, search every move, sample a root child with
 * probability proportional to N^temperature, record (root state, visit policy),
 * and when the sampled child is terminal emit the game's samples with the value
 * signed per player to move (:211-225).  The sink is called once per finished
 * game, in the reference's emission order. */
typedef void (*spai_sample_sink)(void *user, uint32_t game_id, uint32_t n, const float *encodings /* [n][3*6*7] */,
                                 const float *policies /* [n][7] */, const float *values /* [n] */,
                                 const int32_t *moves /* [n] action played at each position */);
typedef struct spai_selfplay_stats {
    double sims;        /* trees x search iterations */
    double evals;       /* leaves sent to the evaluator */
    double games;       /* finished games */
    double positions;   /* emitted samples */
    double moves;       /* search calls (plies of the longest game) */
    double seconds;     /* wall time of the call */
} spai_selfplay_stats;
int spai_selfplay_run(spai_engine *eng, uint32_t n_games, uint64_t game_id_base, spai_sample_sink sink, void *user,
                      spai_selfplay_stats *stats);
/* The same n_games games (ids game_id_base + i, i < n_games; every game's moves,
 * samples and outcome identical to spai_selfplay_run's, the draws keyed by the
 * game id and the game's own move number) played through `window` tree slots:
 * a finished game's slot takes the next game at once, so the device keeps
 * `window` games in flight until the last ones finish instead of searching
 * ever fewer trees as a lockstep batch runs out (the reference's main.rs:169-186
 * keeps the device busy with 6 concurrent workers instead).  The sink sees
 * finished games in the order they finish.  window >= n_games is
 * spai_selfplay_run; window <= max_trees. */
int spai_selfplay_stream(spai_engine *eng, uint32_t n_games, uint32_t window, uint64_t game_id_base,
                         spai_sample_sink sink, void *user, spai_selfplay_stats *stats);

/* ------------------------------------------------------------------ profiling
 * Per-kernel average device time of the last spai_selfplay_run / spai_search
 * call, measured with HIP events on each search chain's stream when enabled.
 * enabled = 1 samples every 4th search iteration; enabled = k > 1 every k-th
 * (each sampled iteration adds six event records per chain). */
int spai_engine_set_timing(spai_engine *eng, int enabled);
/* ms[0] select, ms[1] evaluate (NN forward), ms[2] expand+backup; launches[3] */
int spai_engine_timing(spai_engine *eng, double *avg_ms, double *launches);
/* totals behind spai_engine_timing: summed sampled ms and the work items those
 * launches covered (trees for select/expand, evaluated leaves for the forward) */
int spai_engine_timing_items(spai_engine *eng, double *total_ms, double *items);
/* Diagnostic build-in: one forward over `count` random positions with s_memtime
 * stamps at every phase boundary of the fused kernel.  cycles[k] (k < 20) = mean
 * shader cycles from group start to stamp k (0 start, 1 stem, 2..13 residual
 * convs, 14 head conv, 15 linears, 16 end; 17/18/19 = block 0 conv1 k-loop end,
 * epilogue end, barrier passed).  Wall clock (s_memrealtime): cycles[20] = shader
 * cycles from kernel entry to the first group's start, [21] the same in ns, [22] ns
 * from the first group's start to the workgroup's end, [23] ns from the earliest
 * entry to the latest end over the launch.  cycles holds 24 doubles (48 in the
 * k-step diagnostic build, SPAI_DIAG_KSTEP: [24 + ks] after k-step ks of block 1
 * conv 1, [42] before its barrier, [43] after it, [44] its start).  Needs the
 * diagnostic build (SPAI_DIAG); the production library returns
 * SPAI_ERR_UNSUPPORTED.  Never on the timed path. */
int spai_net_phase_cycles(spai_net *net, uint32_t count, double *cycles);
/* Device time of the search's forward launch ALONE (nothing else on the GPU):
 * ms = mean over `iters` back-to-back launches on `count` random reachable
 * positions, HIP events on the engine stream.  Measurement only. */
int spai_net_bench(spai_net *net, uint32_t count, uint32_t iters, double *ms);
/* the same with the group size the search picks when `conc` search chains'
 * forwards share the CUs (conc 1 = spai_net_bench): the timed region's
 * configuration of a chain's forward, measured alone */
int spai_net_bench_conc(spai_net *net, uint32_t count, uint32_t iters, int conc, double *ms);

/* ---------------------------------------------------------------- learner
 * The training step of the C4 net on the device:
 * ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85) = forward in
 * train mode (BatchNorm batch statistics, running statistics with momentum
 * 0.1), loss -(log_softmax(p)·pi).sum()/B + MSE(v, z) (model/mod.rs:128-135),
 * backward, and one Adam step (tch Adam::default(), lr 1e-3, model/mod.rs:107).
 * Parameters use spai_net_create's flat construction order, so
 * spai_learner_params() feeds spai_net_create() for the self-play replicas.
 * With a communicator (spai_learner_set_comm) each rank's mean gradient is
 * weighted by its share of the global batch (B_rank / sum B) and summed over
 * ranks with RCCL, so a step equals one step on the union of the ranks'
 * batches whatever their sizes; BatchNorm batch statistics stay per rank (DDP
 * without SyncBN) and the running statistics are averaged, so the replicas
 * stay identical. */
typedef struct spai_learner spai_learner;
typedef struct spai_adam_config {
    float lr;            /* 1e-3 */
    float beta1, beta2;  /* 0.9, 0.999 */
    float eps;           /* 1e-8 */
    float bn_momentum;   /* 0.1 */
    float bn_eps;        /* 1e-5 */
} spai_adam_config;
#define SPAI_COMM_ID_BYTES 128

int spai_adam_config_default(spai_adam_config *cfg);
int spai_learner_create(spai_engine *eng, int blocks, int hidden, const float *params, size_t n_params,
                        const spai_adam_config *cfg /* NULL = defaults */, spai_learner **out);
int spai_learner_destroy(spai_learner *l);
/* one optimizer step on n samples: states [n][3][6][7] (spai_encode layout),
 * policies [n][7], values [n]; loss[3] = total, policy, value (may be NULL) */
int spai_learner_train_batch(spai_learner *l, uint32_t n, const float *states, const float *policies,
                             const float *values, float *loss);
/* k consecutive train steps of n samples each (step j reads rows [j n, (j+1) n)
 * of the arrays): the same as k spai_learner_train_batch calls, with one host
 * synchronisation at the end (the next batch is staged while a step runs;
 * measured no faster than k single calls: the step is GPU-bound);
 * losses[3 k] = each step's total, policy, value (may be NULL) */
int spai_learner_train_batches(spai_learner *l, uint32_t k, uint32_t n, const float *states, const float *policies,
                               const float *values, float *losses);
/* Model::train (model/mod.rs:100-149): a fresh Adam, one random permutation of
 * the n samples (keyed by seed), then `epochs` passes of ceil(n / batch) train
 * steps (the last batch may be short); loss[3] = the last step's */
int spai_learner_train(spai_learner *l, uint32_t n, const float *states, const float *policies, const float *values,
                       uint32_t epochs, uint32_t batch, uint64_t seed, float *loss);
/* current parameters (incl. BN running statistics) / last step's gradients
 * (after the cross-rank reduction, before the 1/world scale), flat order */
int spai_learner_params(spai_learner *l, float *params, size_t n_params);
int spai_learner_grads(spai_learner *l, float *grads, size_t n_params);
/* the last train step's post-ReLU activations of conv layer `layer` (stem, the
 * 2*blocks residual convs, policy head, value head), [B][co][6][7]: the ReLU
 * masks the step took, for checking gradients against a float64 restatement */
int spai_learner_activation(spai_learner *l, int layer, float *out, size_t n);
/* RCCL communicator for a data-parallel learner: rank 0 makes the id
 * (spai_comm_unique_id), the host side broadcasts it, every rank joins.
 * world 1 with an id builds a 1-rank communicator (the all-reduce is then a
 * copy); world 1 with NULL drops the communicator. */
int spai_comm_unique_id(uint8_t *id /* SPAI_COMM_ID_BYTES */);
int spai_learner_set_comm(spai_learner *l, int rank, int world, const uint8_t *id);
/* A stand-alone RCCL communicator, one rank per GPU (comm.cpp).  The worker
 * fan-out it sits beside (main.rs:169-186,220-234) has no collective: the
 * sharded self-play bench reduces its per-rank work counters and step times
 * through it once per run, so an N-GPU run shows RCCL formed N ranks over
 * xGMI.  RCCL refuses two ranks on one device: such ranks use the host group.
 * spai_comm_allreduce_f64 reduces n host doubles in place (H2D, ncclAllReduce,
 * D2H on the communicator's stream; blocks until every rank has arrived). */
typedef struct spai_comm spai_comm;
enum { SPAI_REDUCE_SUM = 0, SPAI_REDUCE_MAX = 1 };
int spai_comm_create(int device, int rank, int world, const uint8_t *id /* SPAI_COMM_ID_BYTES */,
                     spai_comm **out);
int spai_comm_allreduce_f64(spai_comm *c, double *buf, size_t n, int op /* SPAI_REDUCE_* */);
int spai_comm_info(spai_comm *c, int *rank, int *world, int *device);
int spai_comm_destroy(spai_comm *c);
/* Weight refresh for self-play replicas (learner_concurrent.rs:158-159,260-264 hands the
 * trainer's weights to the self-play workers): RCCL broadcast of rank `root`'s parameters
 * to every rank of the communicator; a learner without one is left unchanged. */
int spai_learner_broadcast(spai_learner *l, int root);
/* Host collective in place of RCCL, for ranks that cannot form an RCCL
 * communicator (several ranks on one device, a host process group):
 * fn(user, buf, n) must sum the n floats of buf element-wise over the `world`
 * ranks in place (the same rank order on every rank, so the replicas stay
 * bit-identical) and return 0.  The step runs the same batch-size weighting and
 * running-statistic averaging as with RCCL; each all-reduce is staged through
 * pinned host memory and the call blocks in fn until every rank has arrived.
 * spai_learner_broadcast then sums rank `root`'s parameters with -0.0 from every
 * other rank (x + -0.0 == x for every x).  fn NULL (or world 1) drops it;
 * setting one drops an RCCL communicator and vice versa. */
typedef int (*spai_host_allreduce)(void *user, float *buf, size_t n);
int spai_learner_set_host_comm(spai_learner *l, int rank, int world, spai_host_allreduce fn, void *user);
/* the batch size of the latest train step (0 before the first); after
 * spai_learner_train it is the last minibatch's (n % batch, or batch) */
int spai_learner_last_batch(spai_learner *l, uint32_t *n);

/* ---------------------------------------------------------------- checkpoints
 * safetensors files with tch VarStore naming (VarStore::save / load,
 * learner.rs:192, main.rs:61): the flat construction-order parameters <-> one
 * F32 tensor per variable ("weight", "bias", "weight__2", ... "running_var__5"
 * ...), shapes as tch (conv [co][ci][k][k], linear [out][in]).  game = Connect4,
 * TicTacToe (hidden 64) or chess (hidden 256; the flat layout of
 * spai_chess_net_init_params).  Host-only: no device needed. */
int spai_params_save_safetensors(int game, int blocks, int hidden, const float *params, size_t n_params,
                                 const char *path);
int spai_params_load_safetensors(int game, int blocks, int hidden, const char *path, float *params,
                                 size_t n_params);

/* ---------------------------------------------------------------- replay + pipeline
 * Replay ring (learner_concurrent.rs:244-290, capacity batch_size*100 in
 * main.rs:142): pushes overwrite the oldest samples (push_iter_overwrite),
 * pops take the oldest n (pop_iter().take(n)).  Samples are one state
 * encoding [3][6][7], a policy [7] and a value.  Host memory, thread-safe. */
typedef struct spai_replay spai_replay;
int spai_replay_create(uint32_t capacity, spai_replay **out);
int spai_replay_destroy(spai_replay *r);
int spai_replay_push(spai_replay *r, uint32_t n, const float *states, const float *policies, const float *values);
/* SPAI_ERR_INVALID when fewer than n samples are buffered (non-blocking) */
int spai_replay_pop(spai_replay *r, uint32_t n, float *states, float *policies, float *values);
int spai_replay_size(spai_replay *r, uint32_t *n);
/* choose_multiple: k distinct indices of [0, n) from the Philox stream (seed, stream) */
int spai_choose_multiple(uint32_t n, uint32_t k, uint64_t seed, uint64_t stream, uint32_t *out);

/* train_concurrent (main.rs:137-235): n_selfplay self-play workers (host
 * threads, one engine each on selfplay_devices[w]) loop while training: take
 * the latest published weights, play games_per_batch games, push a random
 * sample_fraction of the positions into the replay ring.  The learner (on
 * learner_device) runs train_iters x batches_per_iter train steps of
 * batch_size popped samples, then publishes its weights and, if
 * checkpoint_dir is set, saves {checkpoint_dir}/{iter}.safetensors.
 * Reference defaults (SelfPlayArgs / TrainingArgs / C4 Args): c 2, 600 sims,
 * T 1.25, 100 games, batch 128, 20 batches x 10 iters, capacity 12800,
 * fraction 0.3, 4 blocks.
 *
 * Optional observer (cfg.observer, NULL = none): called under the replay ring's
 * lock, so the events arrive in ring order.  A PUSH event carries a worker's
 * subsample (n = (positions as f32 * fraction) as usize, learner_concurrent.rs:278)
 * and the weight version its games were played with; a POP event carries the
 * batch the trainer took for one train step and the number of weight versions
 * published so far.  Tests replay the events through a HeapRb model.  The
 * callback must not call back into the pipeline.  It runs while the ring's lock
 * is held, so every self-play worker and the trainer wait for it: it must be
 * fast and must not block (copy what it needs and return); run timings with an
 * observer are not representative. */
enum { SPAI_PIPE_PUSH = 0, SPAI_PIPE_POP = 1 };
typedef struct spai_pipeline_event {
    int32_t kind;          /* SPAI_PIPE_PUSH / SPAI_PIPE_POP */
    uint32_t worker;       /* push: worker index; pop: 0 */
    uint64_t batch;        /* push: the worker's self-play batch number; pop: train step */
    uint64_t version;      /* push: weight version played with; pop: versions published */
    uint32_t n;            /* samples pushed / popped */
    uint32_t positions;    /* push: positions of the self-play batch; pop: 0 */
    uint32_t ring_size;    /* samples buffered after the event */
    uint32_t pad;
    const float *states, *policies, *values;   /* [n][126], [n][7], [n] */
} spai_pipeline_event;
typedef void (*spai_pipeline_observer)(void *user, const spai_pipeline_event *ev);
typedef struct spai_pipeline_config {
    /* ABI guard: the caller sets struct_size = sizeof(spai_pipeline_config) before
     * spai_pipeline_config_default / spai_pipeline_run; a size the library was not
     * built with (a client compiled against another header) is refused with
     * SPAI_ERR_INVALID before anything is read or written (added in 0.2 with the
     * observer fields) */
    uint32_t struct_size;
    uint32_t n_selfplay;
    const int *selfplay_devices;   /* [n_selfplay] */
    int learner_device;
    uint32_t games_per_batch, num_searches;
    float c, temperature;
    uint32_t batch_size, batches_per_iter, train_iters, replay_capacity;
    float sample_fraction;
    int blocks;
    uint64_t seed;
    const char *checkpoint_dir;    /* NULL: no checkpoints */
    spai_pipeline_observer observer;   /* NULL: no events */
    void *observer_user;
} spai_pipeline_config;
typedef struct spai_pipeline_stats {
    double games, positions, samples_pushed, samples_overwritten, batches_trained;
    double last_loss[3];
    double weight_version_published, weight_version_used_max, seconds;
} spai_pipeline_stats;
int spai_pipeline_config_default(spai_pipeline_config *cfg);
int spai_pipeline_run(const spai_pipeline_config *cfg, const float *init_params, size_t n_params,
                      spai_pipeline_stats *stats);


/* ---------------------------------------------------------------- chess
 * game/chess.rs (the adapter over the `chess` crate 3.2.0) on the device:
 * config 4 of BASELINE.json.  A separate engine type: a position is a set of
 * bitboards, a move is a 16-bit code, the policy has 73*8*8 = 4672 entries
 * (chess.rs:252-257), the encoding is [19][8][8] (chess.rs:176-249).
 *
 * Move code: src | dst << 6 | promo << 12; squares rank*8 + file (a1 = 0);
 * promo = 1 knight, 2 bishop, 3 rook, 4 queen (chess::Piece index), 0 none.
 * Move lists are in MoveGen::new_legal enumeration order (piece type P, N, B,
 * R, Q, K; unpinned sources before pinned ones; en-passant captures after the
 * pawns; destinations ascending; promotions Q, N, R, B).  The reference's
 * repetition count compares these ordered lists (chess.rs:51-61); the device
 * compares 64-bit hashes of them. */
#define SPAI_CHESS_POLICY 4672
#define SPAI_CHESS_ENC 1216
#define SPAI_CHESS_MAX_MOVES 256

typedef struct spai_chess_state {
    uint64_t pieces[6];   /* Pawn, Knight, Bishop, Rook, Queen, King (chess::Piece order) */
    uint64_t colors[2];   /* White, Black */
    uint8_t side;         /* 0 White to move, 1 Black */
    uint8_t castle;       /* 1 white kingside, 2 white queenside, 4 black kingside, 8 black queenside */
    uint8_t ep;           /* chess::Board::en_passant: square of the pawn that just double-pushed, 64 = none */
    uint8_t status;       /* spai_status (filled by reads) */
    uint16_t fifty;       /* fifty_move_rule_halfmove_counter (chess.rs:29) */
    uint16_t made;        /* Action::MakeMove count of the Game (chess.rs:243-246) */
    uint32_t reps;        /* get_num_repetitions (chess.rs:51-61; filled by reads) */
    uint32_t pad;
} spai_chess_state;

typedef struct spai_chess spai_chess;
typedef struct spai_chess_net spai_chess_net;

/* cfg.max_moves = longest game (sizes the transposition tables).  Default 12,304: the
 * fifty-move counter (reset by pawn moves, captures and at most 4 castle-rights
 * changes) bounds a game at 12,298 plies, so the default covers every legal game. */
int spai_chess_config_default(spai_config *cfg);
int spai_chess_create(const spai_config *cfg, int device, spai_chess **out);
int spai_chess_destroy(spai_chess *e);
int spai_chess_sync(spai_chess *e);

/* rules over n engine-held slots, each with its own transposition table */
int spai_chess_games_resize(spai_chess *e, uint32_t n);                  /* n x State::default() */
int spai_chess_games_write(spai_chess *e, uint32_t first, uint32_t n, const spai_chess_state *s); /* empty table */
int spai_chess_games_read(spai_chess *e, uint32_t first, uint32_t n, spai_chess_state *s);
/* get_valid_actions (chess.rs:148): moves [n][SPAI_CHESS_MAX_MOVES], counts [n] */
int spai_chess_legal_moves(spai_chess *e, uint32_t first, uint32_t n, uint16_t *moves, uint32_t *counts);
/* get_next_state (chess.rs:108-146) in place: rc SPAI_ERR_GAME_OVER ("Game is already
 * over") or SPAI_ERR_ILLEGAL_MOVE ("Failed to make move"); the slot is unchanged on error */
int spai_chess_apply(spai_chess *e, uint32_t first, uint32_t n, const uint16_t *moves, int32_t *rc);
/* get_status (chess.rs:150-166) and get_num_repetitions; get_value_and_terminated
 * (chess.rs:168-174: Won -> +1, quirk Q7).  Any output may be NULL. */
int spai_chess_status(spai_chess *e, uint32_t first, uint32_t n, uint8_t *status, uint32_t *reps, float *value,
                      uint8_t *terminated);
/* get_encoding: out [n][19][8][8] f32 */
int spai_chess_encode(spai_chess *e, uint32_t first, uint32_t n, float *out);
/* Device time (HIP events, mean of iters launches) of the batched rules kernels
 * over slots [first, first+n): ms[0] legal move lists + counts + status,
 * ms[1] encoding.  Measurement only; slots are not modified. */
int spai_chess_rules_bench(spai_chess *e, uint32_t first, uint32_t n, uint32_t iters, double *ms);
/* perft of slot `slot`'s position on the device: counts[d-1] = the number of legal
 * move sequences of length d, d = 1..depth (<= 8), by the movegen and make-move
 * the search uses (MoveGen::new_legal / Board::make_move of the chess crate,
 * game/chess.rs:54,117-118); breadth first, one Board array per ply in HBM
 * (SPAI_ERR_CAPACITY past 2^26 positions in one ply) */
int spai_chess_perft(spai_chess *e, uint32_t slot, int depth, uint64_t *counts);
/* mask_invalid_actions (chess.rs:252-275): policy [n][len] -> out [n][4672]; len must be 4672 */
int spai_chess_mask_invalid(spai_chess *e, uint32_t first, uint32_t n, const float *policy, uint32_t len,
                            float *out);
/* Policy::get_prob / set_prob flat index of a move (get_channel, chess.rs:311-393) */
int spai_chess_move_index(int side, uint16_t move, int32_t *index);
/* Policy::get_action (chess.rs:395-493), including its knight-underpromotion bug (:442) */
int spai_chess_index_move(int side, int32_t index, uint16_t *move);

/* net: model/chess.rs:48-77 (torso = stem + `blocks` residual blocks of 256
 * channels; policy head conv1x1 256->256 + ReLU + conv1x1 256->73; value head
 * conv1x1 256->1 + ReLU + linear 64->256 + ReLU + linear 256->1 + tanh).  params
 * in tch construction order as for spai_net_create.  bf16 MFMA, fp32 accumulate. */
int spai_chess_net_num_params(int blocks, size_t *count);
int spai_chess_net_init_params(int blocks, uint64_t seed, float *params);
int spai_chess_net_create(spai_chess *e, int blocks, const float *params, size_t n_params, spai_chess_net **out);
int spai_chess_net_destroy(spai_chess_net *net);
/* Net::forward(x, train=false): x [n][19][8][8] -> logits [n][4672], value [n] */
int spai_chess_net_forward(spai_chess_net *net, uint32_t n, const float *x, float *logits, float *value);
/* Model::predict (model/mod.rs:36-98) over game slots [first, first+n): encoding
 * (with each slot's repetition count), forward, softmax, mask_invalid_actions ->
 * priors [n][4672], values [n]; all on the device. */
int spai_chess_predict(spai_chess_net *net, uint32_t first, uint32_t n, float *priors, float *values);
int spai_chess_set_net(spai_chess *e, spai_chess_net *net);

/* search: Tree (mcts.rs) + Mcts::search over chess trees held on the device.
 * Per tree i: policy [i][4672] normalized root visits (NULL allowed),
 * child_ids / child_visits / child_moves [i][SPAI_CHESS_MAX_MOVES], n_children [i]. */
int spai_chess_trees_create(spai_chess *e, uint32_t n);                   /* n x Tree::default() */
int spai_chess_search(spai_chess *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                      uint32_t *child_ids, float *child_visits, uint16_t *child_moves, uint32_t *n_children);
/* Tree::use_subtree for the k-th root child (k in [0, n_children)); the new root keeps N and W */
/* Tree::with_root_state (mcts.rs:86-89): tree `tree` becomes a one-node tree rooted at the
 * state held in game slot `slot` (board, MakeMove count, fifty-move counter and the slot's
 * history of earlier positions, which the repetition rule reads) */
int spai_chess_tree_reset(spai_chess *e, uint32_t tree, uint32_t slot);
int spai_chess_tree_use_subtree(spai_chess *e, uint32_t tree, uint32_t child_index);
int spai_chess_tree_root(spai_chess *e, uint32_t tree, spai_chess_state *root, uint32_t *visits, float *value_sum);
/* use_subtree for n trees at once (child_index[i] of tree_idx[i]'s root children); status[i] /
 * reps[i] = get_status / get_num_repetitions of the new root (either may be NULL) */
int spai_chess_trees_advance(spai_chess *e, uint32_t n, const uint32_t *tree_idx, const uint32_t *child_index,
                             uint8_t *status, uint32_t *reps);

/* SelfPlayWorker::self_play (learner_concurrent.rs:169-242) for chess */
typedef void (*spai_chess_sample_sink)(void *user, uint32_t game_id, uint32_t n,
                                       const float *encodings /* [n][19*64] */,
                                       const float *policies /* [n][4672] */, const float *values /* [n] */,
                                       const uint16_t *moves /* [n] move played at each position */);
int spai_chess_selfplay_run(spai_chess *e, uint32_t n_games, uint64_t game_id_base, spai_chess_sample_sink sink,
                            void *user, spai_selfplay_stats *stats);
/* The same n_games chess games played through `window` tree slots (window <=
 * max_trees), a finished game's slot taking the next game at once; every game
 * identical to spai_chess_selfplay_run's (draws keyed by game id and the game's
 * own move number), the sink sees games in the order they finish. */
int spai_chess_selfplay_stream(spai_chess *e, uint32_t n_games, uint32_t window, uint64_t game_id_base,
                               spai_chess_sample_sink sink, void *user, spai_selfplay_stats *stats);
/* timing of the last search / self-play call, as spai_engine_timing:
 * ms[0] select + leaf rules, ms[1] net forward, ms[2] expand + backup */
int spai_chess_set_timing(spai_chess *e, int enabled);
int spai_chess_timing(spai_chess *e, double *avg_ms, double *launches, double *items);


/* ---------------------------------------------------------------- tictactoe
 * game/tictactoe.rs + model/tictactoe.rs (BASELINE config 1) on the device.
 * Board = two 9-bit masks, bit row*3 + col (the flat action index of the
 * row-major 3x3 Policy, tictactoe.rs:100-102); X moves first; X to move iff
 * num_actions_played is even.  Same conventions as the Connect4 entry points;
 * the net is fp32 (hidden 64) and the policy has 9 entries. */
typedef struct spai_ttt_state {
    uint16_t x, o;
    uint8_t num_actions_played, status;
    uint8_t pad[2];
} spai_ttt_state;
typedef struct spai_ttt spai_ttt;
typedef struct spai_ttt_net spai_ttt_net;
int spai_ttt_create(const spai_config *cfg, int device, spai_ttt **out);
int spai_ttt_destroy(spai_ttt *e);
int spai_ttt_games_resize(spai_ttt *e, uint32_t n);
int spai_ttt_games_write(spai_ttt *e, uint32_t first, uint32_t n, const spai_ttt_state *s);
int spai_ttt_games_read(spai_ttt *e, uint32_t first, uint32_t n, spai_ttt_state *s);
int spai_ttt_legal_mask(spai_ttt *e, uint32_t first, uint32_t n, uint32_t *mask);        /* tictactoe.rs:169-182 */
int spai_ttt_apply(spai_ttt *e, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc);  /* :127-167 */
int spai_ttt_encode(spai_ttt *e, uint32_t first, uint32_t n, float *out);                /* [n][3][3][3], :199-216 */
int spai_ttt_mask_invalid(spai_ttt *e, uint32_t first, uint32_t n, const float *policy, uint32_t len,
                          float *out);                                                   /* :218-236, len 9 */
int spai_ttt_net_num_params(int blocks, size_t *count);
int spai_ttt_net_init_params(int blocks, uint64_t seed, float *params);
int spai_ttt_net_create(spai_ttt *e, int blocks, const float *params, size_t n_params, spai_ttt_net **out);
int spai_ttt_net_destroy(spai_ttt_net *net);
int spai_ttt_net_forward(spai_ttt_net *net, uint32_t n, const float *x, float *logits, float *value);
/* Model::predict over game slots [first, first+n) -> priors [n][9], values [n] */
int spai_ttt_predict(spai_ttt_net *net, uint32_t first, uint32_t n, float *priors, float *values);
int spai_ttt_set_net(spai_ttt *e, spai_ttt_net *net);
int spai_ttt_trees_create(spai_ttt *e, uint32_t n);
/* per tree i: policy [i][9], child_ids / child_visits [i][9], n_children [i] (any may be NULL) */
int spai_ttt_search(spai_ttt *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                    uint32_t *child_ids, float *child_visits, uint32_t *n_children);
/* Tree::with_root_state (mcts.rs:86-89) */
int spai_ttt_tree_reset(spai_ttt *e, uint32_t tree, const spai_ttt_state *root);
int spai_ttt_tree_use_subtree(spai_ttt *e, uint32_t tree, uint32_t child_index);
/* SelfPlayWorker::self_play; the sink gets encodings [n][27], policies [n][9], values, moves */
int spai_ttt_selfplay_run(spai_ttt *e, uint32_t n_games, uint64_t game_id_base, spai_sample_sink sink, void *user,
                          spai_selfplay_stats *stats);
/* the same games through `window` tree slots (spai_selfplay_stream's contract) */
int spai_ttt_selfplay_stream(spai_ttt *e, uint32_t n_games, uint32_t window, uint64_t game_id_base,
                             spai_sample_sink sink, void *user, spai_selfplay_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
