//! Drop-in replacement for the reference's src/model/connect_four.rs.
//!
//! `Net::new` builds the same tch modules in the same order as
//! model/connect_four.rs:50-72 (so the VarStore, its checkpoints and the
//! trainer's `forward(x, true)` are unchanged), and keeps shallow handles to
//! every variable in construction order.  Inference runs on the MI355X:
//! `forward(x, false)` and the search (`Net::search_trees`) go through libspai
//! with a device copy of the weights, rebuilt whenever the VarStore's values
//! change (the trainer -> self-play weight copy of learner_concurrent.rs:158-159
//! needs no extra call).  bf16 MFMA by default; SPAI_DTYPE=f32 selects the
//! reference's fp32 arithmetic.
use std::sync::Mutex;

use tch::nn::{self, ModuleT, SequentialT};
use tch::{Device, Kind, Tensor};

use crate::game::connect_four::{self, State as C4State};
use crate::game::{Policy as _, State as _};
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

/// engine + device net for this Net, created on first use
struct Gpu {
    engine: *mut sys::spai_engine,
    net: *mut sys::spai_net,
    max_trees: u32,
    num_searches: u32,
    fingerprint: Option<u64>,
}
// the handles are used by one thread at a time (one engine per self-play worker, main.rs:169-186)
unsafe impl Send for Gpu {}

impl Drop for Gpu {
    fn drop(&mut self) {
        unsafe {
            if !self.net.is_null() {
                sys::spai_net_destroy(self.net);
            }
            if !self.engine.is_null() {
                sys::spai_engine_destroy(self.engine);
            }
        }
    }
}

/// the device learner for this Net (engine + spai_learner), created on the first
/// train step from the VarStore's values; its Adam moments persist across steps
/// like the trainer's tch optimizer (learner_concurrent.rs:42-48)
struct Trainer {
    engine: *mut sys::spai_engine,
    learner: *mut sys::spai_learner,
    n_params: usize,
    // VarStore fingerprint after the learner's last write-back: a different one
    // means the trainer's variables were changed from outside (VarStore::load /
    // copy), and the learner is rebuilt from them rather than overwriting them
    fingerprint: Option<u64>,
}
unsafe impl Send for Trainer {}

impl Drop for Trainer {
    fn drop(&mut self) {
        unsafe {
            if !self.learner.is_null() {
                sys::spai_learner_destroy(self.learner);
            }
            if !self.engine.is_null() {
                sys::spai_engine_destroy(self.engine);
            }
        }
    }
}

pub struct Net {
    torso: SequentialT,
    policy_head: SequentialT,
    value_head: SequentialT,
    blocks: u32,
    vars: Vec<Tensor>,   // construction (= spai_net_create flat) order
    dev: Mutex<Option<Gpu>>,
    trainer: Mutex<Option<Trainer>>,
}

fn conv_bn(vs: &nn::Path, ci: i64, co: i64, vars: &mut Vec<Tensor>) -> (nn::Conv2D, nn::BatchNorm) {
    let conv = nn::conv2d(vs, ci, co, 3, nn::ConvConfig { padding: 1, ..Default::default() });
    let bn = nn::batch_norm2d(vs, co, Default::default());
    vars.push(conv.ws.shallow_clone());
    vars.push(conv.bs.as_ref().unwrap().shallow_clone());
    vars.push(bn.ws.as_ref().unwrap().shallow_clone());
    vars.push(bn.bs.as_ref().unwrap().shallow_clone());
    vars.push(bn.running_mean.shallow_clone());
    vars.push(bn.running_var.shallow_clone());
    (conv, bn)
}

fn linear(vs: &nn::Path, i: i64, o: i64, vars: &mut Vec<Tensor>) -> nn::Linear {
    let l = nn::linear(vs, i, o, Default::default());
    vars.push(l.ws.shallow_clone());
    vars.push(l.bs.as_ref().unwrap().shallow_clone());
    l
}

impl super::Net for Net {
    type State = connect_four::State;
    type Args = Args;

    // model/connect_four.rs:50-72 with model/mod.rs:152-184 (new_resnet) inlined in the same order
    fn new(vs: &nn::Path, args: Args) -> Self {
        let (blocks, h) = (args.num_resnet_blocks, args.num_hidden);
        let mut vars = Vec::new();
        let (c, b) = conv_bn(vs, 3, h, &mut vars);
        let mut torso = nn::seq_t().add_fn(|x| x.view((-1, 3, 6, 7))).add(c).add(b).add_fn(|x| x.relu());
        for _ in 0..blocks {
            let (c1, b1) = conv_bn(vs, h, h, &mut vars);
            let (c2, b2) = conv_bn(vs, h, h, &mut vars);
            let seq = nn::seq_t().add(c1).add(b1).add_fn(|x| x.relu()).add(c2).add(b2);
            torso = torso.add(nn::func_t(move |x, train| (x + x.apply_t(&seq, train)).relu()));
        }
        let (pc, pb) = conv_bn(vs, h, 32, &mut vars);
        let pl = linear(vs, 32 * 6 * 7, 7, &mut vars);
        let policy_head = nn::seq_t().add(pc).add(pb).add_fn(|x| x.relu()).add_fn(|x| x.flat_view()).add(pl);
        let (vc, vb) = conv_bn(vs, h, 3, &mut vars);
        let vl = linear(vs, 3 * 6 * 7, 1, &mut vars);
        let value_head = nn::seq_t().add(vc).add(vb).add_fn(|x| x.relu()).add_fn(|x| x.flat_view()).add(vl)
            .add_fn(|x| x.tanh());
        assert_eq!(h, 64, "the device net is built for 64 hidden channels");
        Self { torso, policy_head, value_head, blocks, vars, dev: Mutex::new(None), trainer: Mutex::new(None) }
    }

    // train = true: the tch graph (the trainer's autograd path, model/mod.rs:100-149);
    // train = false: Net::forward on the device (spai_net_forward)
    fn forward(&self, x: &Tensor, train: bool) -> (Tensor, Tensor) {
        if train {
            let t = self.torso.forward_t(x, true);
            return (self.policy_head.forward_t(&t, true), self.value_head.forward_t(&t, true));
        }
        let n = x.size()[0];
        let xs = Vec::<f32>::try_from(x.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        let mut logits = vec![0f32; n as usize * 7];
        let mut value = vec![0f32; n as usize];
        let mut g = self.device(0, None);   // any engine: forward does not touch the trees
        let d = g.as_mut().unwrap();
        sys::check(unsafe { sys::spai_net_forward(d.net, n as u32, xs.as_ptr(), logits.as_mut_ptr(), value.as_mut_ptr()) });
        (Tensor::from_slice(&logits).view((n, 7)).to_device(x.device()),
         Tensor::from_slice(&value).view((n, 1)).to_device(x.device()))
    }

    fn search_trees(&self, args: &MctsArgs, trees: &mut [&mut Tree<C4State>])
        -> Vec<super::SearchResult<C4State>> {
        self.device_search(args, trees)
    }

    fn device_train_batch(&self, states: &Tensor, policies: &Tensor, values: &Tensor) -> Option<f64> {
        Some(self.device_train(states, policies, values))
    }
}

impl Net {
    /// one device train step (spai_learner_train_batch, fp32 on the exact-f32 MFMA),
    /// then the VarStore variables (and through them the trainer's checkpoints and
    /// the self-play weight copy, learner_concurrent.rs:155-161) take the new values
    fn device_train(&self, states: &Tensor, policies: &Tensor, values: &Tensor) -> f64 {
        let flat = |t: &Tensor| Vec::<f32>::try_from(t.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        let (x, pi, z) = (flat(states), flat(policies), flat(values));
        let n = z.len();
        assert!(x.len() == n * 126 && pi.len() == n * 7, "train batch shapes: [n][3][6][7], [n][7], [n](x1)");
        let mut g = self.trainer.lock().unwrap();
        if g.as_ref().map_or(false, |t| t.fingerprint != Some(self.fingerprint())) {
            *g = None;   // Drop destroys the stale learner and its engine
        }
        if g.is_none() {
            let mut cfg = sys::spai_config::default();
            sys::check(unsafe { sys::spai_config_default(sys::SPAI_GAME_CONNECT4, &mut cfg) });
            cfg.max_trees = 1;
            cfg.num_searches = 1;
            let device = std::env::var("SPAI_TRAIN_DEVICE").or_else(|_| std::env::var("SPAI_DEVICE")).ok()
                .and_then(|v| v.parse().ok()).unwrap_or(0);
            let mut e = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_engine_create(sys::SPAI_GAME_CONNECT4, &cfg, device, &mut e) });
            let p = self.params();
            let mut l = std::ptr::null_mut();
            sys::check(unsafe {
                sys::spai_learner_create(e, self.blocks as i32, 64, p.as_ptr(), p.len(), std::ptr::null(), &mut l)
            });
            *g = Some(Trainer { engine: e, learner: l, n_params: p.len(), fingerprint: None });
        }
        let t = g.as_mut().unwrap();
        let mut loss = [0f32; 3];
        sys::check(unsafe {
            sys::spai_learner_train_batch(t.learner, n as u32, x.as_ptr(), pi.as_ptr(), z.as_ptr(), loss.as_mut_ptr())
        });
        let mut p = vec![0f32; t.n_params];
        sys::check(unsafe { sys::spai_learner_params(t.learner, p.as_mut_ptr(), p.len()) });
        let _guard = tch::no_grad_guard();
        let mut off = 0usize;
        for v in &self.vars {
            let k = v.numel();
            let src = Tensor::from_slice(&p[off..off + k]).view(v.size().as_slice()).to_device(v.device());
            v.shallow_clone().copy_(&src);
            off += k;
        }
        assert_eq!(off, p.len(), "VarStore variables vs the device learner's flat parameters");
        t.fingerprint = Some(self.fingerprint());
        loss[0] as f64
    }
}

impl Net {
    fn params(&self) -> Vec<f32> {
        let mut p = Vec::new();
        for t in &self.vars {
            let v = Vec::<f32>::try_from(t.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
            p.extend_from_slice(&v);
        }
        p
    }

    /// bit-exact fingerprint of the VarStore's values (model/mod.rs `fingerprint`: panics
    /// on a NaN or infinite parameter, so a diverged model is reported rather than the
    /// device learner being rebuilt, and its Adam state reset, on every step)
    fn fingerprint(&self) -> u64 {
        super::fingerprint(&self.vars)
    }

    /// the device engine (at least `trees` trees; `num_searches` per search, None =
    /// whatever the engine has) and a device net holding the current VarStore values
    fn device(&self, trees: u32, num_searches: Option<u32>) -> std::sync::MutexGuard<'_, Option<Gpu>> {
        let mut g = self.dev.lock().unwrap();
        let fp = self.fingerprint();
        let stale = match g.as_ref() {
            None => true,
            Some(d) => d.max_trees < trees || num_searches.map_or(false, |s| s != d.num_searches),
        };
        let num_searches = num_searches.unwrap_or(1);
        if stale {
            *g = None;   // drop the old engine first
            let mut cfg = sys::spai_config::default();
            sys::check(unsafe { sys::spai_config_default(sys::SPAI_GAME_CONNECT4, &mut cfg) });
            cfg.max_trees = trees.max(1);
            cfg.num_searches = num_searches;
            cfg.eval = sys::SPAI_EVAL_NET;
            let device = std::env::var("SPAI_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0);
            let mut e = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_engine_create(sys::SPAI_GAME_CONNECT4, &cfg, device, &mut e) });
            *g = Some(Gpu { engine: e, net: std::ptr::null_mut(), max_trees: cfg.max_trees, num_searches,
                                fingerprint: None });
        }
        let d = g.as_mut().unwrap();
        if d.net.is_null() || d.fingerprint != Some(fp) {
            let p = self.params();
            let dtype = if std::env::var("SPAI_DTYPE").as_deref() == Ok("f32") { sys::SPAI_DTYPE_F32 } else { sys::SPAI_DTYPE_BF16 };
            let mut net = std::ptr::null_mut();
            sys::check(unsafe { sys::spai_net_create(d.engine, self.blocks as i32, 64, p.as_ptr(), p.len(), dtype, &mut net) });
            if !d.net.is_null() {
                unsafe { sys::spai_net_destroy(d.net) };
            }
            d.net = net;
            d.fingerprint = Some(fp);
            sys::check(unsafe { sys::spai_engine_set_net(d.engine, net) });
        }
        g
    }
}

impl Net {
    // Mcts::search (mcts.rs:196-332) for Connect4 trees, all on the device
    fn device_search(&self, args: &MctsArgs, trees: &mut [&mut Tree<C4State>])
        -> Vec<(connect_four::Policy, Vec<(usize, f32)>)> {
        let n = trees.len();
        if n == 0 {
            return Vec::new();
        }
        let fresh = trees.iter().all(|t| t.binding.is_none());
        let mut g = self.device(if fresh { n as u32 } else { 0 }, Some(args.num_searches));
        let d = g.as_mut().unwrap();
        let engine = d.engine as usize;
        if fresh {   // a new batch of trees: slots 0..n, roots uploaded
            sys::check(unsafe { sys::spai_trees_create(d.engine, n as u32) });
            for (slot, t) in trees.iter_mut().enumerate() {
                t.binding = Some(DeviceBinding { engine, game: sys::SPAI_GAME_CONNECT4, slot: slot as u32 });
                if t.pending_root || t.arena[0].state != C4State::default() {
                    let root = t.arena[0].state.to_ffi();
                    sys::check(unsafe { sys::spai_tree_reset(d.engine, slot as u32, &root) });
                }
                t.pending_root = false;
            }
        }
        assert!(trees.iter().all(|t| t.binding.map(|b| b.engine) == Some(engine)),
                "a search batch mixes trees of different engines / batches");
        let idx: Vec<u32> = trees.iter().map(|t| t.binding.unwrap().slot).collect();
        let mut pol = vec![0f32; n * 7];
        let mut ids = vec![0u32; n * 7];
        let mut vis = vec![0f32; n * 7];
        let mut nch = vec![0u32; n];
        sys::check(unsafe {
            sys::spai_search(d.engine, n as u32, idx.as_ptr(), args.num_searches, pol.as_mut_ptr(), ids.as_mut_ptr(),
                             vis.as_mut_ptr(), nch.as_mut_ptr())
        });
        let mut out = Vec::with_capacity(n);
        for (i, t) in trees.iter_mut().enumerate() {
            let root = t.arena[0].state.clone();
            let actions = root.get_valid_actions();
            let k = nch[i] as usize;
            let mut children = Vec::with_capacity(k);
            let mut child_probs = Vec::with_capacity(k);
            let mut visits = connect_four::Policy::default();
            for j in 0..k {
                let a = actions[j].clone();
                visits.set_prob(&a, vis[i * 7 + j]);
                children.push(Node {
                    state: root.get_next_state(&a).unwrap(),
                    action_taken: Some(a),
                    visit_count: vis[i * 7 + j] as u32,
                    device_id: ids[i * 7 + j],
                    ..Default::default()
                });
                child_probs.push((j + 1, vis[i * 7 + j]));
            }
            visits.normalize();   // Policy::normalize of the root visit counts (mcts.rs:318-328)
            t.set_root_children(children);
            out.push((visits, child_probs));
        }
        out
    }
}
