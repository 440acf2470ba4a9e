//! Raw bindings of include/spai.h (the C ABI of libspai.so) used by the drop-in
//! modules in this directory.  Every function returns 0 or a negative spai_error;
//! `check` turns a failure into the reference's behaviour, a panic with the
//! library's message (the reference `unwrap()`s every Result on this path).
#![allow(non_camel_case_types, dead_code)]
use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};

pub const SPAI_GAME_TICTACTOE: c_int = 0;
pub const SPAI_GAME_CONNECT4: c_int = 1;
pub const SPAI_GAME_CHESS: c_int = 2;
pub const SPAI_EVAL_NET: u32 = 0;
pub const SPAI_DTYPE_BF16: c_int = 0;
pub const SPAI_DTYPE_F32: c_int = 1;
pub const SPAI_ERR_ILLEGAL_MOVE: c_int = -2;
pub const SPAI_ERR_GAME_OVER: c_int = -3;
pub const SPAI_CHESS_POLICY: usize = 4672;
pub const SPAI_CHESS_MAX_MOVES: usize = 256;

#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct spai_c4_state {
    pub x: u64,
    pub o: u64,
    pub num_actions_played: u8,
    pub status: u8,
    pub pad: [u8; 6],
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct spai_ttt_state {
    pub x: u16,
    pub o: u16,
    pub num_actions_played: u8,
    pub status: u8,
    pub pad: [u8; 2],
}

/// spai_chess_state (include/spai.h): bitboards in chess::Piece / Color order
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct spai_chess_state {
    pub pieces: [u64; 6],
    pub colors: [u64; 2],
    pub side: u8,
    pub castle: u8,
    pub ep: u8,
    pub status: u8,
    pub fifty: u16,
    pub made: u16,
    pub reps: u32,
    pub pad: u32,
}

impl spai_chess_state {
    /// the start position (chess::Game::new(), game/chess.rs:94-101)
    pub fn start() -> Self {
        Self {
            pieces: [0x00FF_0000_0000_FF00, 0x4200_0000_0000_0042, 0x2400_0000_0000_0024, 0x8100_0000_0000_0081,
                     0x0800_0000_0000_0008, 0x1000_0000_0000_0010],
            colors: [0xFFFF, 0xFFFF_0000_0000_0000],
            side: 0,
            castle: 15,
            ep: 64,
            ..Default::default()
        }
    }
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct spai_config {
    pub c: f32,
    pub num_searches: u32,
    pub temperature: f32,
    pub max_trees: u32,
    pub max_moves: u32,
    pub eval: u32,
    pub seed: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct spai_selfplay_stats {
    pub sims: f64,
    pub evals: f64,
    pub games: f64,
    pub positions: f64,
    pub moves: f64,
    pub seconds: f64,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct spai_adam_config {
    pub lr: f32,
    pub beta1: f32,
    pub beta2: f32,
    pub eps: f32,
    pub bn_momentum: f32,
    pub bn_eps: f32,
}

pub enum spai_engine {}
pub enum spai_net {}
pub enum spai_learner {}
pub enum spai_ttt {}
pub enum spai_ttt_net {}
pub enum spai_chess {}
pub enum spai_chess_net {}

pub type spai_sample_sink = extern "C" fn(
    user: *mut c_void,
    game_id: u32,
    n: u32,
    encodings: *const f32,
    policies: *const f32,
    values: *const f32,
    moves: *const i32,
);

#[link(name = "spai")]
extern "C" {
    pub fn spai_last_error() -> *const c_char;
    pub fn spai_config_default(game: c_int, cfg: *mut spai_config) -> c_int;
    pub fn spai_engine_create(game: c_int, cfg: *const spai_config, device: c_int, out: *mut *mut spai_engine) -> c_int;
    pub fn spai_engine_destroy(e: *mut spai_engine) -> c_int;

    // Net trait + Model::predict (model/mod.rs:22-98)
    pub fn spai_net_num_params(game: c_int, blocks: c_int, hidden: c_int, count: *mut usize) -> c_int;
    pub fn spai_net_create(e: *mut spai_engine, blocks: c_int, hidden: c_int, params: *const f32, n: usize,
                           dtype: c_int, out: *mut *mut spai_net) -> c_int;
    pub fn spai_net_destroy(net: *mut spai_net) -> c_int;
    pub fn spai_net_forward(net: *mut spai_net, n: u32, x: *const f32, logits: *mut f32, value: *mut f32) -> c_int;
    pub fn spai_predict(net: *mut spai_net, n: u32, states: *const spai_c4_state, priors: *mut f32,
                        values: *mut f32) -> c_int;
    pub fn spai_engine_set_net(e: *mut spai_engine, net: *mut spai_net) -> c_int;

    // Tree + Mcts::search (mcts.rs:32-39,67-89,161-192,196-332)
    pub fn spai_trees_create(e: *mut spai_engine, n: u32) -> c_int;
    pub fn spai_tree_reset(e: *mut spai_engine, tree: u32, root: *const spai_c4_state) -> c_int;
    pub fn spai_search(e: *mut spai_engine, n: u32, tree_idx: *const u32, num_searches: u32, policy: *mut f32,
                       child_ids: *mut u32, child_visits: *mut f32, n_children: *mut u32) -> c_int;
    pub fn spai_tree_use_subtree(e: *mut spai_engine, tree: u32, child_id: u32) -> c_int;
    pub fn spai_selfplay_run(e: *mut spai_engine, n_games: u32, game_id_base: u64, sink: spai_sample_sink,
                             user: *mut c_void, stats: *mut spai_selfplay_stats) -> c_int;
    pub fn spai_selfplay_stream(e: *mut spai_engine, n_games: u32, window: u32, game_id_base: u64,
                                sink: spai_sample_sink, user: *mut c_void, stats: *mut spai_selfplay_stats) -> c_int;

    // TicTacToe (game/tictactoe.rs, model/tictactoe.rs)
    pub fn spai_ttt_create(cfg: *const spai_config, device: c_int, out: *mut *mut spai_ttt) -> c_int;
    pub fn spai_ttt_destroy(e: *mut spai_ttt) -> c_int;
    pub fn spai_ttt_net_create(e: *mut spai_ttt, blocks: c_int, params: *const f32, n: usize,
                               out: *mut *mut spai_ttt_net) -> c_int;
    pub fn spai_ttt_net_destroy(net: *mut spai_ttt_net) -> c_int;
    pub fn spai_ttt_net_forward(net: *mut spai_ttt_net, n: u32, x: *const f32, logits: *mut f32, value: *mut f32)
        -> c_int;
    pub fn spai_ttt_set_net(e: *mut spai_ttt, net: *mut spai_ttt_net) -> c_int;
    pub fn spai_ttt_trees_create(e: *mut spai_ttt, n: u32) -> c_int;
    pub fn spai_ttt_tree_reset(e: *mut spai_ttt, tree: u32, root: *const spai_ttt_state) -> c_int;
    pub fn spai_ttt_search(e: *mut spai_ttt, n: u32, tree_idx: *const u32, num_searches: u32, policy: *mut f32,
                           child_ids: *mut u32, child_visits: *mut f32, n_children: *mut u32) -> c_int;
    pub fn spai_ttt_tree_use_subtree(e: *mut spai_ttt, tree: u32, child_index: u32) -> c_int;

    // chess (game/chess.rs, model/chess.rs): game slots, net, trees
    pub fn spai_chess_config_default(cfg: *mut spai_config) -> c_int;
    pub fn spai_chess_create(cfg: *const spai_config, device: c_int, out: *mut *mut spai_chess) -> c_int;
    pub fn spai_chess_destroy(e: *mut spai_chess) -> c_int;
    pub fn spai_chess_games_resize(e: *mut spai_chess, n: u32) -> c_int;
    pub fn spai_chess_games_write(e: *mut spai_chess, first: u32, n: u32, s: *const spai_chess_state) -> c_int;
    pub fn spai_chess_games_read(e: *mut spai_chess, first: u32, n: u32, s: *mut spai_chess_state) -> c_int;
    pub fn spai_chess_apply(e: *mut spai_chess, first: u32, n: u32, moves: *const u16, rc: *mut i32) -> c_int;
    pub fn spai_chess_net_create(e: *mut spai_chess, blocks: c_int, params: *const f32, n: usize,
                                 out: *mut *mut spai_chess_net) -> c_int;
    pub fn spai_chess_net_destroy(net: *mut spai_chess_net) -> c_int;
    pub fn spai_chess_net_forward(net: *mut spai_chess_net, n: u32, x: *const f32, logits: *mut f32, value: *mut f32)
        -> c_int;
    pub fn spai_chess_set_net(e: *mut spai_chess, net: *mut spai_chess_net) -> c_int;
    pub fn spai_chess_trees_create(e: *mut spai_chess, n: u32) -> c_int;
    pub fn spai_chess_tree_reset(e: *mut spai_chess, tree: u32, slot: u32) -> c_int;
    pub fn spai_chess_search(e: *mut spai_chess, n: u32, tree_idx: *const u32, num_searches: u32, policy: *mut f32,
                             child_ids: *mut u32, child_visits: *mut f32, child_moves: *mut u16,
                             n_children: *mut u32) -> c_int;
    pub fn spai_chess_tree_use_subtree(e: *mut spai_chess, tree: u32, child_index: u32) -> c_int;

    // Policy trait helpers on a flat policy (game/mod.rs:35-44)
    pub fn spai_policy_normalize(p: *mut f32, n: u32) -> c_int;
    pub fn spai_policy_best_action(p: *const f32, n: u32, index: *mut u32) -> c_int;
    pub fn spai_policy_sample(p: *const f32, n: u32, temperature: f32, u01: f32, index: *mut u32) -> c_int;

    // learner (ModelTrainerWorker::train_batch, learner_concurrent.rs:72-85)
    pub fn spai_adam_config_default(cfg: *mut spai_adam_config) -> c_int;
    pub fn spai_learner_create(e: *mut spai_engine, blocks: c_int, hidden: c_int, params: *const f32, n: usize,
                               cfg: *const spai_adam_config, out: *mut *mut spai_learner) -> c_int;
    pub fn spai_learner_destroy(l: *mut spai_learner) -> c_int;
    pub fn spai_learner_train_batch(l: *mut spai_learner, n: u32, states: *const f32, policies: *const f32,
                                    values: *const f32, loss: *mut f32) -> c_int;
    pub fn spai_learner_params(l: *mut spai_learner, params: *mut f32, n: usize) -> c_int;
    pub fn spai_comm_unique_id(id: *mut u8) -> c_int;
    pub fn spai_learner_set_comm(l: *mut spai_learner, rank: c_int, world: c_int, id: *const u8) -> c_int;
    pub fn spai_learner_broadcast(l: *mut spai_learner, root: c_int) -> c_int;
    pub fn spai_learner_set_host_comm(l: *mut spai_learner, rank: c_int, world: c_int,
                                      f: Option<extern "C" fn(*mut c_void, *mut f32, usize) -> c_int>,
                                      user: *mut c_void) -> c_int;
    pub fn spai_learner_last_batch(l: *mut spai_learner, n: *mut u32) -> c_int;

    // checkpoints (VarStore::save / load: learner.rs:192, main.rs:61)
    pub fn spai_params_save_safetensors(game: c_int, blocks: c_int, hidden: c_int, params: *const f32, n: usize,
                                        path: *const c_char) -> c_int;
    pub fn spai_params_load_safetensors(game: c_int, blocks: c_int, hidden: c_int, path: *const c_char,
                                        params: *mut f32, n: usize) -> c_int;
}

/// The library's message for the last failure on this thread.
pub fn last_error() -> String {
    unsafe { CStr::from_ptr(spai_last_error()).to_string_lossy().into_owned() }
}

/// `rc == 0` or panic with the library's message (the reference unwrap()s).
pub fn check(rc: c_int) {
    if rc != 0 {
        panic!("spai error {}: {}", rc, last_error());
    }
}
