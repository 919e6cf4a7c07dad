// Flow definition tabs with a list + settings layout: Info (info/infoSettingsContent.jsx), Reference data
// (referenceData/*), Functions (function/*: UDF / UDAF / Azure Function, plus the GPU-native HIP UDF / UDAF),
// Scale (scale/scaleSettingsContent.jsx: GPUs instead of executors) and Schedule (schedule/*: recurring and
// one-time batch windows for batching mode).
import { h } from '../common/dom.js';
import { TextField, Dropdown, Toggle, Slider, ItemList, StatementBox, Button, functionEnabled } from '../common/components.js';
import * as Models from './models.js';
import * as V from './validation.js';

const idError = v => (V.isNumberAndStringOnly(v || '') ? null : 'letters and digits only');

// ---- Info ------------------------------------------------------------------------------------------------------
export function InfoTab(flow, ui) {
    return h(
        'div',
        null,
        TextField('Flow display name', flow.displayName, v => { flow.displayName = v; ui.touch(); }, {
            disabled: !functionEnabled('flowNameTextboxEnabled'),
            validate: v => (v && v.trim() ? null : 'a display name is required')
        }),
        TextField('Flow name (derived from the display name on first save)', flow.name || '(not saved yet)', () => null, { disabled: true }),
        TextField('Owner', flow.owner, v => { flow.owner = v; ui.touch(); }),
        StatementBox('i', 'A flow reads one input, projects it (normalization snippet), runs the SQL of the Query tab ' +
            'and the rules on the GPU each micro-batch, and writes the OUTPUT tables to the sinks of the Outputs tab.')
    );
}

// ---- generic list + editor layout -------------------------------------------------------------------------------
function listEditor(ui, key, items, labelOf, isValid, onAdd, onDelete, editor, opts) {
    opts = opts || {};
    let sel = ui.selected[key] || 0;
    if (sel >= items.length) sel = ui.selected[key] = Math.max(0, items.length - 1);
    return h(
        'div',
        { class: 'cols' },
        ItemList(
            items,
            sel,
            labelOf,
            i => { ui.selected[key] = i; ui.update(); },
            onAdd,
            onDelete,
            {
                isValid,
                addDisabled: opts.addDisabled,
                deleteDisabled: opts.deleteDisabled,
                canDelete: opts.canDelete || (() => true),
                addMenu: opts.addMenu
            }
        ),
        h('div', { class: 'grow' }, items.length ? editor(items[sel], sel) : h('div', { class: 'muted' }, opts.empty || 'Nothing here yet.'))
    );
}

function addMenu(types, onAdd, disabled) {
    const sel = h('select', { disabled }, types.map(t => h('option', { value: t.key }, t.name)));
    return h('div', { class: 'row' }, sel, Button('+ Add', () => onAdd(sel.value), { disabled }));
}

// ---- Reference data ----------------------------------------------------------------------------------------------
export function ReferenceDataTab(flow, ui) {
    const items = flow.referenceData;
    return h(
        'div',
        null,
        StatementBox('i', 'Reference tables are loaded once per job (rank 0 reads, an RCCL broadcast shares them) and ' +
            'kept in HBM for joins; use their id as a table name in the query.'),
        listEditor(
            ui,
            'referenceData',
            items,
            r => r.id || '(new)',
            V.isReferenceDataComplete,
            () => {
                items.push(Models.defaultReferenceData());
                ui.selected.referenceData = items.length - 1;
                ui.touch();
                ui.update();
            },
            i => { items.splice(i, 1); ui.touch(); ui.update(); },
            r =>
                h(
                    'div',
                    null,
                    Dropdown('Type', Models.referenceDataTypes, r.type, v => { r.type = v; ui.touch(); }),
                    TextField('Alias (table name)', r.id, v => { r.id = v; ui.touch(); }, { validate: idError }),
                    TextField('Path (local path, file://, wasbs:// or keyvault://)', r.properties.path, v => { r.properties.path = v; ui.touch(); }),
                    Dropdown('Delimiter', Models.csvDelimiters, r.properties.delimiter, v => { r.properties.delimiter = v; ui.touch(); }),
                    Toggle('First row is a header', r.properties.header, v => { r.properties.header = v; ui.touch(); })
                ),
            {
                addDisabled: !functionEnabled('addReferenceDataButtonEnabled'),
                deleteDisabled: !functionEnabled('deleteReferenceDataButtonEnabled'),
                empty: 'No reference data.'
            }
        )
    );
}

// ---- Functions -------------------------------------------------------------------------------------------------
function functionEditor(f, ui) {
    const p = f.properties;
    const head = [
        h('div', { class: 'muted' }, Models.functionTypes.find(t => t.key === f.type).name),
        TextField('Alias (name used in SQL)', f.id, v => { f.id = v; ui.touch(); }, { validate: idError })
    ];
    if (f.type === 'hipUDF' || f.type === 'hipUDAF') {
        return h(
            'div',
            null,
            head,
            TextField(
                f.type === 'hipUDF' ? 'HIP source: a __device__ scalar function' : 'HIP source: State + init / update / merge / finish',
                p.source,
                v => { p.source = v; ui.touch(); },
                { multiline: true, mono: true, height: '180px' }
            ),
            f.type === 'hipUDF'
                ? TextField('Entry function (default: the alias)', p.entry, v => { p.entry = v; ui.touch(); })
                : TextField('Function name prefix', p.prefix, v => { p.prefix = v; ui.touch(); }),
            Dropdown('Return type', Models.udfValueTypes, p.returnType, v => { p.returnType = v; ui.touch(); }),
            TextField('Argument types (comma separated)', (p.argTypes || []).join(','), v => {
                p.argTypes = v.split(',').map(x => x.trim()).filter(Boolean);
                ui.touch();
            }),
            Toggle('Null-safe (called for null arguments too)', p.nullSafe, v => { p.nullSafe = v; ui.touch(); }),
            StatementBox('i', 'Compiled with hipRTC for gfx950 at job start and fused into the query\'s generated kernel.')
        );
    }
    if (f.type === 'azureFunction') {
        return h(
            'div',
            null,
            head,
            TextField('Service endpoint', p.serviceEndpoint, v => { p.serviceEndpoint = v; ui.touch(); }),
            TextField('API name', p.api, v => { p.api = v; ui.touch(); }),
            TextField('Function key (stored as a secret)', p.code, v => { p.code = v; ui.touch(); }, { type: 'password' }),
            Dropdown('Method', Models.functionMethodTypes, p.methodType, v => { p.methodType = v; ui.touch(); }),
            TextField('Parameters (comma separated)', (p.params || []).join(','), v => {
                p.params = v.split(',').map(x => x.trim()).filter(Boolean);
                ui.touch();
            })
        );
    }
    return h(
        'div',
        null,
        head,
        TextField('Module path', p.path, v => { p.path = v; ui.touch(); }),
        TextField('Class name', p.class, v => { p.class = v; ui.touch(); }),
        TextField('Extra library paths (comma separated)', (p.libs || []).join(','), v => {
            p.libs = v.split(',').map(x => x.trim()).filter(Boolean);
            ui.touch();
        })
    );
}

export function FunctionsTab(flow, ui) {
    const items = flow.functions;
    const disabled = !functionEnabled('addFunctionButtonEnabled');
    return listEditor(
        ui,
        'functions',
        items,
        f => `${f.id || '(new)'} · ${f.type}`,
        V.isFunctionComplete,
        () => null,
        i => { items.splice(i, 1); ui.touch(); ui.update(); },
        f => functionEditor(f, ui),
        {
            addMenu: addMenu(Models.functionTypes, t => {
                items.push(Models.defaultFunction(t));
                ui.selected.functions = items.length - 1;
                ui.touch();
                ui.update();
            }, disabled),
            deleteDisabled: !functionEnabled('deleteFunctionButtonEnabled'),
            empty: 'No functions.'
        }
    );
}

// ---- Scale -----------------------------------------------------------------------------------------------------
export function ScaleTab(flow, ui) {
    const s = flow.scale;
    return h(
        'div',
        null,
        Slider('GPUs (one process per MI355X, RCCL over xGMI between them)', s.jobNumGpus || '1', 1, 8, v => {
            s.jobNumGpus = String(v);
            ui.touch();
        }, { disabled: !functionEnabled('scaleGpusSliderEnabled') }),
        StatementBox('i', 'Each GPU holds 288 GB of HBM3E: window panes, state tables and reference data stay resident. ' +
            'Inputs are split across ranks by partition (Kafka / Event Hubs) or by file; keyed SQL shuffles rows over RCCL.')
    );
}

// ---- Schedule ----------------------------------------------------------------------------------------------------
function batchEditor(b, ui) {
    const p = b.properties;
    const f = (label, key, opts) => TextField(label, p[key], v => { p[key] = v; ui.touch(); }, opts);
    const unit = (label, key) => Dropdown(label, Models.batchIntervalTypes, p[key], v => { p[key] = v; ui.touch(); });
    return h(
        'div',
        null,
        h('div', { class: 'muted' }, b.type === 'oneTime' ? 'One-time batch over a fixed time range' : 'Recurring batch'),
        TextField('Id', b.id, v => { b.id = v; ui.touch(); }, { validate: idError }),
        h('div', { class: 'row' }, f('Interval', 'interval'), unit('unit', 'intervalType')),
        b.type === 'recurring' ? h('div', { class: 'row' }, f('Delay', 'delay'), unit('unit', 'delayType')) : null,
        h('div', { class: 'row' }, f('Window', 'window'), unit('unit', 'windowType')),
        f('Start time (UTC, ISO 8601)', 'startTime'),
        f('End time (UTC, ISO 8601)' + (b.type === 'oneTime' ? '' : ' — optional'), 'endTime'),
        p.lastProcessedTime ? h('div', { class: 'muted' }, 'Last processed: ' + p.lastProcessedTime) : null,
        Toggle('Disabled', b.disabled, v => { b.disabled = v; ui.touch(); })
    );
}

export function ScheduleTab(flow, ui) {
    if (flow.input.mode !== 'batching') {
        return StatementBox('i', 'Schedules apply to batching flows; switch the input mode to Batching on the Input tab.');
    }
    const items = flow.batchList;
    const disabled = !functionEnabled('addBatchButtonEnabled');
    return listEditor(
        ui,
        'batchList',
        items,
        b => `${b.id || '(new)'} · ${b.type}${b.disabled ? ' (disabled)' : ''}`,
        V.isBatchComplete,
        () => null,
        i => { items.splice(i, 1); ui.touch(); ui.update(); },
        b => batchEditor(b, ui),
        {
            addMenu: addMenu(Models.batchTypes, t => {
                const b = Models.defaultBatch(t);
                b.id = 'batch' + (items.length + 1);
                items.push(b);
                ui.selected.batchList = items.length - 1;
                ui.touch();
                ui.update();
            }, disabled),
            deleteDisabled: !functionEnabled('deleteBatchButtonEnabled'),
            empty: 'No batch schedule yet.'
        }
    );
}
