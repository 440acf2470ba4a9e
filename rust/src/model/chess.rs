//! Drop-in replacement for the reference's src/model/chess.rs (BASELINE config 4)
//! over the chess engine of libspai (`spai_chess_*`).
//!
//! `Net::new` builds the reference's tch modules in the reference's order
//! (model/chess.rs:48-70: resnet torso on 19 input planes; policy head conv1x1
//! h -> 256 + ReLU + conv1x1 256 -> 73, flattened; value head conv1x1 h -> 1 +
//! ReLU + linear 64 -> 256 + ReLU + linear 256 -> 1 + tanh), so the VarStore and
//! its checkpoints are unchanged and `forward(x, true)` trains on tch.
//! `forward(x, false)` and the search run on the device (bf16 MFMA net,
//! `spai_chess_net_forward` / `spai_chess_search`).
//!
//! game/chess.rs is the reference's, unchanged.  Its State keeps the game as a
//! `chess::Game` whose action list is public, so a root crosses the C ABI by
//! replaying that game's moves from the start position in a device game slot
//! (`spai_chess_apply`): the slot then holds the same board, MakeMove count,
//! fifty-move counter and transposition table (the legal-move lists of every
//! earlier position, chess.rs:51-61,118-146) as the State, and the tree is rooted
//! there (`spai_chess_tree_reset`).  The replayed board is checked against
//! `game.current_position()`; a State that does not descend from `Game::new()`
//! (State::default, chess.rs:94-101) is refused with a panic.
use std::sync::Mutex;

use chess::{Action as GameAction, ChessMove, Color, File, Piece, Rank, Square, ALL_PIECES};
use tch::nn::{self, ModuleT, SequentialT};
use tch::{Device, Kind, Tensor};

use crate::game::chess::State as ChessState;
use crate::game::{Policy as _, State as _};
use crate::mcts::{Args as MctsArgs, DeviceBinding, Node, Tree};
use crate::mcts::spai_sys as sys;

pub struct Args {
    pub num_resnet_blocks: u32,
    pub num_hidden: i64,
}

impl Default for Args {
    fn default() -> Self {
        Self { num_resnet_blocks: 10, num_hidden: 256 }
    }
}

struct Gpu {
    engine: *mut sys::spai_chess,
    net: *mut sys::spai_chess_net,
    max_trees: u32,
    num_searches: u32,
    fingerprint: Option<u64>,
}
// used by one thread at a time (one Mcts + Model per self-play worker, main.rs:169-186)
unsafe impl Send for Gpu {}

impl Drop for Gpu {
    fn drop(&mut self) {
        unsafe {
            if !self.net.is_null() {
                sys::spai_chess_net_destroy(self.net);
            }
            if !self.engine.is_null() {
                sys::spai_chess_destroy(self.engine);
            }
        }
    }
}

pub struct Net {
    torso: SequentialT,
    policy_head: SequentialT,
    value_head: SequentialT,
    blocks: u32,
    vars: Vec<Tensor>,
    dev: Mutex<Option<Gpu>>,
}

/// the engine's 16-bit move code: src | dst << 6 | promo << 12 (promo = chess::Piece index)
fn move_code(m: &ChessMove) -> u16 {
    let promo = m.get_promotion().map_or(0u16, |p| p.to_index() as u16);
    m.get_source().to_index() as u16 | (m.get_dest().to_index() as u16) << 6 | promo << 12
}

fn square(index: u16) -> Square {
    Square::make_square(Rank::from_index(index as usize / 8), File::from_index(index as usize % 8))
}

fn chess_move(code: u16) -> ChessMove {
    let promo = match (code >> 12) & 7 {
        1 => Some(Piece::Knight),
        2 => Some(Piece::Bishop),
        3 => Some(Piece::Rook),
        4 => Some(Piece::Queen),
        _ => None,
    };
    ChessMove::new(square(code & 63), square((code >> 6) & 63), promo)
}

impl super::Net for Net {
    type State = ChessState;
    type Args = Args;

    fn new(vs: &nn::Path, args: Args) -> Self {
        let (blocks, h) = (args.num_resnet_blocks, args.num_hidden);
        let mut vars = Vec::new();
        let torso = super::resnet_tracked(vs, blocks, 19, h, &mut vars);
        let p1 = super::conv_tracked(vs, h, 256, 1, 0, &mut vars);
        let p2 = super::conv_tracked(vs, 256, 73, 1, 0, &mut vars);
        let policy_head = nn::seq_t().add(p1).add_fn(|x| x.relu()).add(p2).add_fn(|x| x.flat_view());
        let v1 = super::conv_tracked(vs, h, 1, 1, 0, &mut vars);
        let l1 = super::linear_tracked(vs, 8 * 8, 256, &mut vars);
        let l2 = super::linear_tracked(vs, 256, 1, &mut vars);
        let value_head = nn::seq_t().add(v1).add_fn(|x| x.relu()).add_fn(|x| x.flat_view()).add(l1)
            .add_fn(|x| x.relu()).add(l2).add_fn(|x| x.tanh());
        assert_eq!(h, 256, "the device chess net is built for 256 hidden channels");
        Self { torso, policy_head, value_head, blocks, vars, dev: Mutex::new(None) }
    }

    fn forward(&self, x: &Tensor, train: bool) -> (Tensor, Tensor) {
        if train {
            let t = self.torso.forward_t(x, true);
            return (self.policy_head.forward_t(&t, true), self.value_head.forward_t(&t, true));
        }
        let n = x.size()[0];
        let xs = Vec::<f32>::try_from(x.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        let mut logits = vec![0f32; n as usize * sys::SPAI_CHESS_POLICY];
        let mut value = vec![0f32; n as usize];
        let mut g = self.device(0, None);
        let d = g.as_mut().unwrap();
        sys::check(unsafe {
            sys::spai_chess_net_forward(d.net, n as u32, xs.as_ptr(), logits.as_mut_ptr(), value.as_mut_ptr())
        });
        (Tensor::from_slice(&logits).view((n, sys::SPAI_CHESS_POLICY as i64)).to_device(x.device()),
         Tensor::from_slice(&value).view((n, 1)).to_device(x.device()))
    }

    // Mcts::search (mcts.rs:196-332) for chess trees on the device
    fn search_trees(&self, args: &MctsArgs, trees: &mut [&mut Tree<ChessState>]) -> Vec<super::SearchResult<ChessState>> {
        let n = trees.len();
        if n == 0 {
            return Vec::new();
        }
        let fresh = trees.iter().all(|t| t.binding.is_none());
        let mut g = self.device(if fresh { n as u32 } else { 0 }, Some(args.num_searches));
        let d = g.as_mut().unwrap();
        let engine = d.engine as usize;
        if fresh {
            sys::check(unsafe { sys::spai_chess_games_resize(d.engine, n as u32) });
            sys::check(unsafe { sys::spai_chess_trees_create(d.engine, n as u32) });
            for (slot, t) in trees.iter_mut().enumerate() {
                replay_into_slot(d.engine, slot as u32, &t.arena[0].state);
                sys::check(unsafe { sys::spai_chess_tree_reset(d.engine, slot as u32, slot as u32) });
                t.binding = Some(DeviceBinding { engine, game: sys::SPAI_GAME_CHESS, slot: slot as u32 });
                t.pending_root = false;
            }
        }
        assert!(trees.iter().all(|t| t.binding.map(|b| b.engine) == Some(engine)),
                "a search batch mixes trees of different engines / batches");
        let idx: Vec<u32> = trees.iter().map(|t| t.binding.unwrap().slot).collect();
        let m = sys::SPAI_CHESS_MAX_MOVES;
        let (mut ids, mut vis, mut mv, mut nch) = (vec![0u32; n * m], vec![0f32; n * m], vec![0u16; n * m], vec![0u32; n]);
        sys::check(unsafe {
            sys::spai_chess_search(d.engine, n as u32, idx.as_ptr(), args.num_searches, std::ptr::null_mut(),
                                   ids.as_mut_ptr(), vis.as_mut_ptr(), mv.as_mut_ptr(), nch.as_mut_ptr())
        });
        let mut out = Vec::with_capacity(n);
        for (i, t) in trees.iter_mut().enumerate() {
            let root = t.arena[0].state.clone();
            let k = nch[i] as usize;
            let mut visits = root.get_zero_policy();
            let mut children = Vec::with_capacity(k);
            let mut child_probs = Vec::with_capacity(k);
            for j in 0..k {
                let a = chess_move(mv[i * m + j]);   // MoveGen::new_legal order, as the reference's children
                let v = vis[i * m + j];
                visits.set_prob(&a, v);
                children.push(Node {
                    state: root.get_next_state(&a).unwrap(),
                    action_taken: Some(a),
                    visit_count: v as u32,
                    device_id: j as u32,   // spai_chess_tree_use_subtree takes the root-child index
                    ..Default::default()
                });
                child_probs.push((j + 1, v));
            }
            visits.normalize();
            t.set_root_children(children);
            out.push((visits, child_probs));
        }
        out
    }
}

/// game slot `slot` := State::default() followed by the State's moves, checked
/// against the State's board
fn replay_into_slot(e: *mut sys::spai_chess, slot: u32, state: &ChessState) {
    let start = sys::spai_chess_state::start();
    sys::check(unsafe { sys::spai_chess_games_write(e, slot, 1, &start) });
    for action in state.game.actions() {
        if let GameAction::MakeMove(m) = action {
            let code = move_code(m);
            let mut rc = 0i32;
            sys::check(unsafe { sys::spai_chess_apply(e, slot, 1, &code, &mut rc) });
            assert!(rc == 0, "replaying the game's move {} failed ({})", m, rc);
        }
    }
    let mut got = sys::spai_chess_state::default();
    sys::check(unsafe { sys::spai_chess_games_read(e, slot, 1, &mut got) });
    let board = state.game.current_position();
    let same = ALL_PIECES.iter().all(|p| got.pieces[p.to_index()] == board.pieces(*p).0)
        && got.colors[0] == board.color_combined(Color::White).0
        && got.colors[1] == board.color_combined(Color::Black).0
        && got.side == (board.side_to_move() == Color::Black) as u8;
    assert!(same, "chess root does not descend from Game::new(): the device replay reached another board");
}

impl Net {
    fn device(&self, trees: u32, num_searches: Option<u32>) -> std::sync::MutexGuard<'_, Option<Gpu>> {
        let mut g = self.dev.lock().unwrap();
        let fp = super::fingerprint(&self.vars);
        let stale = match g.as_ref() {
            None => true,
            Some(d) => d.max_trees < trees || num_searches.map_or(false, |s| s != d.num_searches),
        };
        let num_searches = num_searches.unwrap_or(1);
        if stale {
            *g = None;
            let mut cfg = sys::spai_config::default();
            sys::check(unsafe { sys::spai_chess_config_default(&mut cfg) });
            cfg.max_trees = trees.max(1);
            cfg.num_searches = num_searches;
            cfg.eval = sys::SPAI_EVAL_NET;
            let mut e = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_chess_create(&cfg, super::device_index(), &mut e) });
            *g = Some(Gpu { engine: e, net: std::ptr::null_mut(), max_trees: cfg.max_trees, num_searches,
                            fingerprint: None });
        }
        let d = g.as_mut().unwrap();
        if d.net.is_null() || d.fingerprint != Some(fp) {
            let p = super::flat_params(&self.vars);
            let mut net = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_chess_net_create(d.engine, self.blocks as i32, p.as_ptr(), p.len(), &mut net) });
            if !d.net.is_null() {
                unsafe { sys::spai_chess_net_destroy(d.net) };
            }
            d.net = net;
            d.fingerprint = Some(fp);
            sys::check(unsafe { sys::spai_chess_set_net(d.engine, net) });
        }
        g
    }
}
