//! Drop-in replacement for the reference's src/game/connect_four.rs.
//!
//! Same public types (Player, State, Action, Policy) and the same trait impls
//! (game/mod.rs:21-44), with the board held as the engine's bitboards so a
//! State crosses the C ABI (`spai_c4_state`) without conversion:
//! bit col*7 + row of `x` / `o` is X's / O's stone, row 0 at the bottom,
//! bit 6 of every column always clear.  The rules are the reference's,
//! including its quirk of ignoring the anti-diagonal (connect_four.rs:164-176:
//! only horizontal, vertical and the (+1 row, +1 col) diagonal win), so the
//! win test is "the mover has a line under shifts {1, 7, 8}" (shift 6 is the
//! anti-diagonal).  Policy keeps the reference's Array1 and forwards normalize /
//! get_best_action / sample to the library's Policy helpers (total_cmp last
//! max; rand 0.8 WeightedIndex<f32> fed the rng's own u32).
use std::fmt;

use ndarray::{Array, Array1, Array3, ArrayView1};
use rand::rngs::ThreadRng;
use rand::RngCore;

use crate::mcts::spai_sys as sys;

#[derive(Clone, Copy, Debug, strum_macros::Display, Default, PartialEq, Eq)]
pub enum Player {
    #[default]
    X,
    O,
}

#[derive(Default, Clone, PartialEq)]
pub struct State {
    x: u64,
    o: u64,
    num_actions_played: u8,
    status: super::Status,
}

#[derive(Clone, Debug)]
pub struct Action(pub usize);

#[derive(Clone, Debug)]
pub struct Policy(Array1<f32>);

impl super::Player for Player {
    fn get_opposite(&self) -> Self {
        match self {
            Player::X => Player::O,
            Player::O => Player::X,
        }
    }
}

// bit 6 of every column is always clear, so no shift wraps a line across columns
fn has_line(b: u64) -> bool {
    // vertical (1), horizontal (7), (+1 row, +1 col) diagonal (8); never 6
    [1u32, 7, 8].iter().any(|&s| {
        let m = b & (b >> s);
        m & (m >> (2 * s)) != 0
    })
}

impl State {
    /// the engine's view of this state (spai_c4_state)
    pub fn to_ffi(&self) -> sys::spai_c4_state {
        sys::spai_c4_state {
            x: self.x,
            o: self.o,
            num_actions_played: self.num_actions_played,
            status: match self.status {
                super::Status::Ongoing => 0,
                super::Status::Tied => 1,
                super::Status::Won => 2,
            },
            pad: [0; 6],
        }
    }

    pub fn from_ffi(s: &sys::spai_c4_state) -> Self {
        State {
            x: s.x,
            o: s.o,
            num_actions_played: s.num_actions_played,
            status: match s.status {
                0 => super::Status::Ongoing,
                1 => super::Status::Tied,
                _ => super::Status::Won,
            },
        }
    }

    fn open_columns(&self) -> u32 {
        let occ = self.x | self.o;
        (0..7).filter(|c| (occ >> (7 * c + 5)) & 1 == 0).fold(0, |m, c| m | (1 << c))
    }
}

impl fmt::Display for State {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        writeln!(f, "Current player: {}", super::State::get_current_player(self))?;
        for row in (0..6).rev() {
            let cells: Vec<String> = (0..7)
                .map(|col| {
                    let b = 1u64 << (col * 7 + row);
                    if self.x & b != 0 { "X" } else if self.o & b != 0 { "O" } else { "-" }.to_string()
                })
                .collect();
            writeln!(f, " {}", cells.join(" | "))?;
        }
        Ok(())
    }
}

impl fmt::Display for Action {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "Row: {}", self.0)
    }
}

impl Default for Policy {
    fn default() -> Self {
        Self(Array::zeros(7))
    }
}

impl super::Policy for Policy {
    type Action = Action;

    fn get_prob(&self, action: &Action) -> f32 {
        self.0[[action.0]]
    }

    fn set_prob(&mut self, action: &Action, prob: f32) {
        self.0[[action.0]] = prob;
    }

    fn normalize(&mut self) {
        let p = self.0.as_slice_mut().unwrap();
        sys::check(unsafe { sys::spai_policy_normalize(p.as_mut_ptr(), p.len() as u32) });
    }

    fn get_flat_ndarray(&self) -> Array1<f32> {
        self.0.clone()
    }

    fn sample(&self, rng: &mut ThreadRng, temperature: f32) -> Action {
        // rand 0.8 UniformFloat<f32>: ((u32 >> 9) as f32) * 2^-23, from the same rng
        let u = (rng.next_u32() >> 9) as f32 * (1.0 / (1u32 << 23) as f32);
        let p = self.0.as_slice().unwrap();
        let mut idx = 0u32;
        sys::check(unsafe { sys::spai_policy_sample(p.as_ptr(), p.len() as u32, temperature, u, &mut idx) });
        Action(idx as usize)
    }

    fn get_best_action(&self) -> Action {
        let p = self.0.as_slice().unwrap();
        let mut idx = 0u32;
        sys::check(unsafe { sys::spai_policy_best_action(p.as_ptr(), p.len() as u32, &mut idx) });
        Action(idx as usize)
    }
}

impl super::State for State {
    type Policy = Policy;
    type Player = Player;

    fn get_current_player(&self) -> Player {
        if self.num_actions_played % 2 == 0 { Player::X } else { Player::O }
    }

    // connect_four.rs:190-211
    fn get_next_state(&self, action: &Action) -> Result<Self, String> {
        if self.status != super::Status::Ongoing {
            return Err("Game has already ended".to_string());
        }
        let col = action.0;
        let occ = self.x | self.o;
        let column = (occ >> (7 * col)) & 0x3F;
        if column == 0x3F {
            return Err("Illegal move: column already filled".to_string());
        }
        let bit = 1u64 << (7 * col + column.count_ones() as usize);
        let mut next = self.clone();
        let mover = if self.get_current_player() == Player::X {
            next.x |= bit;
            next.x
        } else {
            next.o |= bit;
            next.o
        };
        next.num_actions_played += 1;
        if has_line(mover) {
            next.status = super::Status::Won;
        } else if next.num_actions_played == 6 * 7 {
            next.status = super::Status::Tied;
        }
        Ok(next)
    }

    // connect_four.rs:213-225: top cell empty, ascending columns, none once ended
    fn get_valid_actions(&self) -> Vec<Action> {
        if self.status != super::Status::Ongoing {
            return Vec::with_capacity(0);
        }
        let open = self.open_columns();
        (0..7).filter(|c| (open >> c) & 1 == 1).map(Action).collect()
    }

    fn get_status(&self) -> super::Status {
        self.status
    }

    // connect_four.rs:231-240
    fn get_value_and_terminated(&self) -> (f32, bool) {
        match self.status {
            super::Status::Won => (-1.0, true),
            super::Status::Tied => (0.0, true),
            super::Status::Ongoing => (0.0, false),
        }
    }

    // connect_four.rs:242-259: [mine, theirs, empty][row][col]
    fn get_encoding(&self) -> Array3<f32> {
        let (mine, theirs) = if self.get_current_player() == Player::X { (self.x, self.o) } else { (self.o, self.x) };
        let mut e = Array3::zeros((3, 6, 7));
        for row in 0..6 {
            for col in 0..7 {
                let b = 1u64 << (col * 7 + row);
                let plane = if mine & b != 0 { 0 } else if theirs & b != 0 { 1 } else { 2 };
                e[[plane, row, col]] = 1.0;
            }
        }
        e
    }

    // connect_four.rs:261-279: p * mask / sum(p * mask) (ndarray's sum; 0/0 = NaN as the reference)
    fn mask_invalid_actions(&self, policy: ArrayView1<f32>) -> Result<Policy, String> {
        if policy.shape() != [7] {
            return Err(format!("Expected policy shape to be (7,), found {:?}", policy.shape()));
        }
        let mut mask = Array::zeros(7);
        for a in self.get_valid_actions() {
            mask[a.0] = 1.0;
        }
        let mut masked = &policy * &mask;
        masked /= masked.sum();
        Ok(Policy(masked))
    }

    fn get_zero_policy(&self) -> Policy {
        Policy::default()
    }
}
