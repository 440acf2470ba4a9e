//! Drop-in replacement for the reference's src/model/tictactoe.rs (BASELINE
//! config 1) over the TicTacToe engine of libspai (`spai_ttt_*`).
//!
//! `Net::new` builds the reference's tch modules in the reference's order
//! (model/tictactoe.rs:50-72: resnet torso on a [-1, 3, 3, 3] view, policy head
//! conv 32 + BN + ReLU + linear 288 -> 9, value head conv 3 + BN + ReLU + linear
//! 27 -> 1 + tanh), so the VarStore, its names and checkpoints are unchanged and
//! `forward(x, true)` trains on tch.  `forward(x, false)` and the search run on
//! the device (fp32 net, `spai_ttt_net_forward` / `spai_ttt_search`) with a copy
//! of the weights rebuilt whenever the VarStore's values change.
//!
//! game/tictactoe.rs is the reference's, unchanged: a root State crosses the C ABI
//! through the public State trait only -- its encoding (plane 0 = the player to
//! move, 1 = the opponent, tictactoe.rs:199-216), `get_current_player` and
//! `get_status` give the two 9-bit masks (bit row*3 + col) of `spai_ttt_state`.
use std::sync::Mutex;

use tch::nn::{self, ModuleT, SequentialT};
use tch::{Device, Kind, Tensor};

use crate::game::tictactoe::{Action, Player, State as TttState};
use crate::game::{Policy as _, State as _, Status};
use crate::mcts::{Args as MctsArgs, DeviceBinding, Node, Tree};
use crate::mcts::spai_sys as sys;

pub struct Args {
    pub num_resnet_blocks: u32,
    pub num_hidden: i64,
}

impl Default for Args {
    fn default() -> Self {
        Self { num_resnet_blocks: 4, num_hidden: 64 }
    }
}

struct Gpu {
    engine: *mut sys::spai_ttt,
    net: *mut sys::spai_ttt_net,
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
                sys::spai_ttt_net_destroy(self.net);
            }
            if !self.engine.is_null() {
                sys::spai_ttt_destroy(self.engine);
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

/// a reference State as the engine's record
fn to_ffi(s: &TttState) -> sys::spai_ttt_state {
    let enc = s.get_encoding();   // [3][3][3]: mover, opponent, empty
    let (mut mover, mut other) = (0u16, 0u16);
    for row in 0..3 {
        for col in 0..3 {
            let bit = 1u16 << (row * 3 + col);
            if enc[[0, row, col]] == 1.0 {
                mover |= bit;
            }
            if enc[[1, row, col]] == 1.0 {
                other |= bit;
            }
        }
    }
    let (x, o) = match s.get_current_player() {
        Player::X => (mover, other),
        Player::O => (other, mover),
    };
    sys::spai_ttt_state {
        x,
        o,
        num_actions_played: (x | o).count_ones() as u8,
        status: match s.get_status() {
            Status::Ongoing => 0,
            Status::Tied => 1,
            Status::Won => 2,
        },
        pad: [0; 2],
    }
}

impl super::Net for Net {
    type State = TttState;
    type Args = Args;

    fn new(vs: &nn::Path, args: Args) -> Self {
        let (blocks, h) = (args.num_resnet_blocks, args.num_hidden);
        let mut vars = Vec::new();
        let torso = nn::seq_t()
            .add_fn(|x| x.view((-1, 3, 3, 3)))
            .add(super::resnet_tracked(vs, blocks, 3, h, &mut vars));
        let (pc, pb) = super::conv_bn_tracked(vs, h, 32, &mut vars);
        let pl = super::linear_tracked(vs, 32 * 9, 9, &mut vars);
        let policy_head = nn::seq_t().add(pc).add(pb).add_fn(|x| x.relu()).add_fn(|x| x.flat_view()).add(pl);
        let (vc, vb) = super::conv_bn_tracked(vs, h, 3, &mut vars);
        let vl = super::linear_tracked(vs, 3 * 9, 1, &mut vars);
        let value_head =
            nn::seq_t().add(vc).add(vb).add_fn(|x| x.relu()).add_fn(|x| x.flat_view()).add(vl).add_fn(|x| x.tanh());
        assert_eq!(h, 64, "the device TicTacToe net is built for 64 hidden channels");
        Self { torso, policy_head, value_head, blocks, vars, dev: Mutex::new(None) }
    }

    fn forward(&self, x: &Tensor, train: bool) -> (Tensor, Tensor) {
        if train {
            let t = self.torso.forward_t(x, true);
            return (self.policy_head.forward_t(&t, true), self.value_head.forward_t(&t, true));
        }
        let n = x.size()[0];
        let xs = Vec::<f32>::try_from(x.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        let mut logits = vec![0f32; n as usize * 9];
        let mut value = vec![0f32; n as usize];
        let mut g = self.device(0, None);
        let d = g.as_mut().unwrap();
        sys::check(unsafe { sys::spai_ttt_net_forward(d.net, n as u32, xs.as_ptr(), logits.as_mut_ptr(), value.as_mut_ptr()) });
        (Tensor::from_slice(&logits).view((n, 9)).to_device(x.device()),
         Tensor::from_slice(&value).view((n, 1)).to_device(x.device()))
    }

    // Mcts::search (mcts.rs:196-332) for TicTacToe trees on the device
    fn search_trees(&self, args: &MctsArgs, trees: &mut [&mut Tree<TttState>]) -> Vec<super::SearchResult<TttState>> {
        let n = trees.len();
        if n == 0 {
            return Vec::new();
        }
        let fresh = trees.iter().all(|t| t.binding.is_none());
        let mut g = self.device(if fresh { n as u32 } else { 0 }, Some(args.num_searches));
        let d = g.as_mut().unwrap();
        let engine = d.engine as usize;
        if fresh {
            sys::check(unsafe { sys::spai_ttt_trees_create(d.engine, n as u32) });
            for (slot, t) in trees.iter_mut().enumerate() {
                t.binding = Some(DeviceBinding { engine, game: sys::SPAI_GAME_TICTACTOE, slot: slot as u32 });
                let root = to_ffi(&t.arena[0].state);
                sys::check(unsafe { sys::spai_ttt_tree_reset(d.engine, slot as u32, &root) });
                t.pending_root = false;
            }
        }
        assert!(trees.iter().all(|t| t.binding.map(|b| b.engine) == Some(engine)),
                "a search batch mixes trees of different engines / batches");
        let idx: Vec<u32> = trees.iter().map(|t| t.binding.unwrap().slot).collect();
        let (mut ids, mut vis, mut nch) = (vec![0u32; n * 9], vec![0f32; n * 9], vec![0u32; n]);
        sys::check(unsafe {
            sys::spai_ttt_search(d.engine, n as u32, idx.as_ptr(), args.num_searches, std::ptr::null_mut(),
                                 ids.as_mut_ptr(), vis.as_mut_ptr(), nch.as_mut_ptr())
        });
        let mut out = Vec::with_capacity(n);
        for (i, t) in trees.iter_mut().enumerate() {
            let root = t.arena[0].state.clone();
            let actions: Vec<Action> = root.get_valid_actions();   // row-major: the engine's child order
            let k = nch[i] as usize;
            let mut visits = root.get_zero_policy();
            let mut children = Vec::with_capacity(k);
            let mut child_probs = Vec::with_capacity(k);
            for j in 0..k {
                let a = actions[j].clone();
                visits.set_prob(&a, vis[i * 9 + j]);
                children.push(Node {
                    state: root.get_next_state(&a).unwrap(),
                    action_taken: Some(a),
                    visit_count: vis[i * 9 + j] as u32,
                    device_id: j as u32,   // spai_ttt_tree_use_subtree takes the root-child index
                    ..Default::default()
                });
                child_probs.push((j + 1, vis[i * 9 + j]));
            }
            visits.normalize();
            t.set_root_children(children);
            out.push((visits, child_probs));
        }
        out
    }
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
            // mcts.rs:46-59 (c 2, T 1.25); a TicTacToe game lasts at most 9 plies
            let cfg = sys::spai_config { c: 2.0, num_searches, temperature: 1.25, max_trees: trees.max(1), max_moves: 9,
                                         eval: sys::SPAI_EVAL_NET, seed: 0 };
            let mut e = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_ttt_create(&cfg, super::device_index(), &mut e) });
            *g = Some(Gpu { engine: e, net: std::ptr::null_mut(), max_trees: cfg.max_trees, num_searches,
                            fingerprint: None });
        }
        let d = g.as_mut().unwrap();
        if d.net.is_null() || d.fingerprint != Some(fp) {
            let p = super::flat_params(&self.vars);
            let mut net = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_ttt_net_create(d.engine, self.blocks as i32, p.as_ptr(), p.len(), &mut net) });
            if !d.net.is_null() {
                unsafe { sys::spai_ttt_net_destroy(d.net) };
            }
            d.net = net;
            d.fingerprint = Some(fp);
            sys::check(unsafe { sys::spai_ttt_set_net(d.engine, net) });
        }
        g
    }
}
