//! Drop-in replacement for the reference's src/mcts.rs: the same public types
//! (Args, Node, Tree, Mcts) and call surface (mcts.rs:8-89,161,196), with the
//! search running on the MI355X engine (libspai, include/spai.h).
//!
//! What stays on the host is what the callers read: `Tree` keeps its public
//! fields (`arena`, `node_id_to_expand`, `state_history`, `policy_history`,
//! `args`).  After a search, `arena` holds the root (id 0) and its children
//! (ids 1..=k, legal-action order) with their states and visit counts, so the
//! reference's self-play loop (learner_concurrent.rs:178-238) runs unchanged:
//! it reads `tree.arena[0].state`, samples a child id from the returned
//! `(child id, visits)` list, reads `tree.arena[id].state` and calls
//! `tree.use_subtree(id)`.  The full tree lives in HBM; its node ids are the
//! engine's, and `use_subtree` re-roots it there (the root keeps N and W, as
//! the reference's BFS copy does, mcts.rs:161-192).
//!
//! A tree is bound to an engine slot the first time it is searched; a batch of
//! fresh trees (`vec![Tree::default(); n]`, learner_concurrent.rs:173) gets
//! slots 0..n of the net's engine.
use crate::game::{Policy, State};
use crate::model::{Model, Net};

// the C ABI bindings live beside this file (src/spai_sys.rs) so that main.rs's
// module list stays the reference's
#[path = "spai_sys.rs"]
pub mod spai_sys;
use spai_sys as sys;

#[derive(Clone, Copy)]
pub struct Args {
    pub c: f32,
    pub num_searches: u32,
    pub temperature: f32,
    pub num_learn_iters: u32,
    pub num_self_play_iters: u32,
    pub num_parallel_self_play_games: usize,
    pub batch_size: i64,
    pub num_epochs: u32,
}

impl Default for Args {
    fn default() -> Self {
        // mcts.rs:46-59
        Args {
            c: 2.0,
            num_searches: 600,
            temperature: 1.25,
            num_learn_iters: 10,
            num_self_play_iters: 500,
            num_parallel_self_play_games: 100,
            batch_size: 32,
            num_epochs: 4,
        }
    }
}

/// A root or root child as last seen by the host (the engine holds the rest).
/// `device_id` is the engine's node id (Connect4) or root-child index (TicTacToe, chess).
#[derive(Clone, Default)]
pub struct Node<T: State> {
    pub state: T,
    pub action_taken: Option<<<T as State>::Policy as Policy>::Action>,
    pub(crate) id: usize,
    pub(crate) visit_count: u32,
    pub(crate) device_id: u32,
}

/// Where a searched tree lives: an engine handle (spai_engine* for Connect4,
/// spai_ttt* for TicTacToe, spai_chess* for chess) and the tree's slot in it.
#[derive(Clone, Copy, PartialEq, Eq, Debug)]
pub struct DeviceBinding {
    pub engine: usize,
    pub game: i32,
    pub slot: u32,
}

#[derive(Clone)]
pub struct Tree<T: State> {
    pub args: Args,
    pub arena: Vec<Node<T>>,
    pub node_id_to_expand: Option<usize>,
    pub state_history: Vec<T>,
    pub policy_history: Vec<T::Policy>,
    /// the engine slot holding this tree once it has been searched
    pub(crate) binding: Option<DeviceBinding>,
    pub(crate) pending_root: bool,
}

impl<T: State> Default for Tree<T> {
    fn default() -> Self {
        Self {
            args: Args::default(),
            arena: vec![Node::default()],
            node_id_to_expand: None,
            state_history: Vec::new(),
            policy_history: Vec::new(),
            binding: None,
            pending_root: false,
        }
    }
}

impl<T: State> Tree<T> {
    /// Tree::with_root_state (mcts.rs:86-89)
    pub fn with_root_state(state: T) -> Self {
        let root = Node { state, ..Default::default() };
        Self { arena: vec![root], pending_root: true, ..Default::default() }
    }

    /// Tree::use_subtree (mcts.rs:161-192): `new_root_id` is a root-child id from
    /// the last search (1..=k); the engine re-roots the device tree in place.
    pub fn use_subtree(&mut self, new_root_id: usize) {
        assert!(new_root_id >= 1 && new_root_id < self.arena.len(), "use_subtree: {} is not a root child", new_root_id);
        let child = self.arena[new_root_id].clone();
        if let Some(b) = self.binding {
            let rc = unsafe {
                match b.game {
                    sys::SPAI_GAME_CONNECT4 => sys::spai_tree_use_subtree(b.engine as *mut sys::spai_engine, b.slot,
                                                                          child.device_id),
                    sys::SPAI_GAME_CHESS => sys::spai_chess_tree_use_subtree(b.engine as *mut sys::spai_chess, b.slot,
                                                                             child.device_id),
                    _ => sys::spai_ttt_tree_use_subtree(b.engine as *mut sys::spai_ttt, b.slot, child.device_id),
                }
            };
            sys::check(rc);
        }
        self.arena = vec![Node { id: 0, ..child }];
    }

    pub(crate) fn set_root_children(&mut self, children: Vec<Node<T>>) {
        self.arena.truncate(1);
        for (k, mut c) in children.into_iter().enumerate() {
            c.id = k + 1;
            self.arena.push(c);
        }
    }
}

pub struct Mcts<T: Net> {
    pub args: Args,
    pub model: Model<T>,
}

// The device search is a provided method of Net (model/mod.rs), overridden by the
// Connect4, TicTacToe and chess nets, so this impl keeps the reference's bound and
// learner.rs / learner_concurrent.rs compile unchanged.
impl<T: Net> Mcts<T> {
    /// Mcts::search (mcts.rs:196-332): `num_searches` iterations over every tree
    /// on the device, then per tree (normalized root visit policy,
    /// [(root-child id, visits)]) in the trees' order.
    pub fn search(&self, trees: &mut Vec<&mut Tree<T::State>>)
        -> Vec<(<<T as Net>::State as State>::Policy, Vec<(usize, f32)>)> {
        self.model.net.search_trees(&self.args, trees.as_mut_slice())
    }
}
