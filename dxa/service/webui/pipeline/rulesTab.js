// Rules tab (datax-pipeline flowDefinition/components/rule/*: rulesSettingsContent, ruleGeneralSettings,
// queryBuilder, ruleAggregateColumnSettings, rulePivotSettings, ruleAlertSettings, conditionsPreview,
// tagRuleSettings). A tag rule is a tree of condition groups; the SQL it becomes (and an aggregate rule's derived
// aggregates / pivots) is previewed by the control plane's designer model (designer/conditions/sql), the same code
// designer/flow/toconfig runs on save.
import { h, mount } from '../common/dom.js';
import { flowApi } from '../common/api.js';
import { TextField, Dropdown, Toggle, Button, ItemList, StatementBox, functionEnabled } from '../common/components.js';
import * as Models from './models.js';
import * as V from './validation.js';

function operatorsFor(rule, c) {
    if (rule.properties.ruleType === 'AggregateRule' && c.aggregate && c.aggregate !== 'none') return Models.numberOperators;
    return Models.numberOperators.concat(Models.stringOperators);
}

// the condition tree editor (queryBuilder.jsx); `changed` re-previews, `rerender` rebuilds the tree
export function ConditionTree(rule, changed, rerender) {
    const agg = rule.properties.ruleType === 'AggregateRule';
    function group(g, depth, parent, index) {
        return h(
            'div',
            { class: 'cond-group' },
            index > 0 ? Dropdown('', Models.conjunctionTypes, g.conjunction, v => { g.conjunction = v; changed(); }) : null,
            g.conditions.map((c, i) => (c.type === 'group' ? group(c, depth + 1, g, i) : condition(c, g, i))),
            h(
                'div',
                { class: 'row' },
                Button('+ condition', () => { g.conditions.push(Models.defaultCondition()); rerender(); }),
                Button('+ group', () => { g.conditions.push(Models.defaultGroup()); rerender(); }),
                parent ? Button('remove group', () => { parent.conditions.splice(index, 1); rerender(); }) : null
            )
        );
    }
    function condition(c, g, i) {
        return h(
            'div',
            { class: 'row' },
            i > 0 ? Dropdown('', Models.conjunctionTypes, c.conjunction, v => { c.conjunction = v; changed(); }) : h('span', { style: { width: '64px' } }),
            agg ? Dropdown('', Models.conditionAggregateTypes, c.aggregate || 'none', v => { c.aggregate = v; rerender(); }) : null,
            TextField('', c.field, v => { c.field = v; changed(); }, { placeholder: 'column' }),
            Dropdown('', operatorsFor(rule, c), c.operator, v => { c.operator = v; changed(); }),
            TextField('', c.value, v => { c.value = v; changed(); }, { placeholder: 'value' }),
            Button('✕', () => { g.conditions.splice(i, 1); rerender(); }, { title: 'remove condition' })
        );
    }
    return group(rule.properties.conditions, 0, null, 0);
}

function ruleEditor(flow, rule, ui) {
    const p = rule.properties;
    const preview = h('div', { class: 'statement mono' }, '...');
    const treeHost = h('div');
    let timer = null;

    async function refreshPreview() {
        const err = V.conditionsError(p.conditions, p.ruleType);
        try {
            const r = await flowApi.conditionsSql(p.conditions, p.ruleType, p.pivots, p.aggs);
            mount(
                preview,
                h('div', null, h('b', null, 'WHERE / HAVING: '), r.condition || ''),
                p.ruleType === 'AggregateRule' ? h('div', null, h('b', null, 'aggregates: '), (r.aggs || []).join(', ') || '-') : null,
                p.ruleType === 'AggregateRule' ? h('div', null, h('b', null, 'GROUP BY: '), (r.pivots || []).join(', ') || '-') : null,
                err || r.error ? h('div', { class: 'errtext' }, err || r.error) : null
            );
            p.condition = r.condition || '';
        } catch (e) {
            mount(preview, h('span', { class: 'errtext' }, e.message));
        }
    }
    const changed = () => {
        ui.touch();
        clearTimeout(timer);
        timer = setTimeout(refreshPreview, 250);
    };
    const rerender = () => {
        mount(treeHost, ConditionTree(rule, changed, rerender));
        changed();
    };
    rerender();

    const sinkChoices = flow.outputs.filter(o => o.id).map(o => o.id);
    const aggRows = (p.aggs || []).map((a, i) =>
        h(
            'div',
            { class: 'row' },
            Dropdown('', Models.aggregateTypes, a.aggregate, v => { a.aggregate = v; changed(); }),
            TextField('', a.column, v => { a.column = v; changed(); }, { placeholder: 'column' }),
            Button('✕', () => { p.aggs.splice(i, 1); ui.touch(); ui.update(); })
        )
    );
    const pivotRows = (p.pivots || []).map((c, i) =>
        h('div', { class: 'row' }, TextField('', c, v => { p.pivots[i] = v; changed(); }, { placeholder: 'column' }),
            Button('✕', () => { p.pivots.splice(i, 1); ui.touch(); ui.update(); }))
    );

    return h(
        'div',
        null,
        h(
            'div',
            { class: 'row' },
            TextField('Rule id', rule.id, v => { rule.id = v; p.ruleId = v; ui.touch(); }),
            Dropdown('Rule type', Models.ruleSubTypes, p.ruleType, v => { p.ruleType = v; ui.touch(); ui.update(); })
        ),
        TextField('Description', p.ruleDescription, v => { p.ruleDescription = v; ui.touch(); },
            { validate: v => (v && v.trim() ? null : 'a description is required') }),
        h('div', { class: 'row' },
            TextField('Tag column', p.tagName, v => { p.tagName = v; ui.touch(); }),
            TextField('Tag value', p.tag, v => { p.tag = v; ui.touch(); })),
        h('div', { class: 'panel-header' }, 'Conditions'),
        treeHost,
        preview,
        p.ruleType === 'AggregateRule'
            ? h(
                'div',
                null,
                h('div', { class: 'panel-header' }, 'Extra aggregates', Button('+', () => { p.aggs.push({ aggregate: 'AVG', column: '' }); ui.touch(); ui.update(); })),
                aggRows,
                h('div', { class: 'panel-header' }, 'Extra GROUP BY columns', Button('+', () => { p.pivots.push(''); ui.touch(); ui.update(); })),
                pivotRows
            )
            : null,
        h('div', { class: 'panel-header' }, 'Alert'),
        Toggle('Send an alert when the rule fires', p.isAlert, v => { p.isAlert = v; ui.touch(); ui.update(); }),
        p.isAlert
            ? h(
                'div',
                null,
                Dropdown('Severity', Models.severityTypes, p.severity, v => { p.severity = v; ui.touch(); }),
                h('div', { class: 'field' }, h('span', { class: 'label' }, 'Alert sinks'),
                    h('div', { class: 'row' }, sinkChoices.map(id =>
                        Toggle(id, (p.alertSinks || []).includes(id), on => {
                            p.alertSinks = (p.alertSinks || []).filter(x => x !== id);
                            if (on) p.alertSinks.push(id);
                            ui.touch();
                        })))),
                Dropdown('Output template', [{ key: '', name: '(default)' }].concat(flow.outputTemplates.map(t => ({ key: t.id, name: t.id }))),
                    p.outputTemplate || '', v => { p.outputTemplate = v; ui.touch(); })
            )
            : null
    );
}

function templatesEditor(flow, ui) {
    const items = flow.outputTemplates;
    return h(
        'div',
        null,
        h('div', { class: 'panel-header' }, 'Alert output templates',
            Button('+', () => { items.push({ id: 'template' + (items.length + 1), template: '' }); ui.touch(); ui.update(); })),
        items.map((t, i) =>
            h('div', { class: 'panel' },
                h('div', { class: 'row' }, TextField('Id', t.id, v => { t.id = v; ui.touch(); }),
                    Button('Delete', () => { items.splice(i, 1); ui.touch(); ui.update(); })),
                TextField('Template (text with ${column} references)', t.template, v => { t.template = v; ui.touch(); }, { multiline: true, mono: true }))
        )
    );
}

export function RulesTab(flow, ui) {
    const items = flow.rules;
    let sel = Math.min(ui.selected.rules || 0, Math.max(0, items.length - 1));
    return h(
        'div',
        null,
        StatementBox('i', 'Tag rules add a tag column to matching events; aggregate rules evaluate over each batch grouped ' +
            'by the GROUP BY columns. Rules are compiled into the flow\'s SQL and run on the GPU with it.'),
        h(
            'div',
            { class: 'cols' },
            ItemList(items, sel, r => `${r.id || '(new)'} · ${r.properties.ruleType === 'AggregateRule' ? 'aggregate' : 'simple'}`,
                i => { ui.selected.rules = i; ui.update(); },
                () => {
                    const r = Models.defaultRule();
                    r.id = r.properties.ruleId = 'rule' + (items.length + 1);
                    r.properties.productId = flow.name;
                    items.push(r);
                    ui.selected.rules = items.length - 1;
                    ui.touch();
                    ui.update();
                },
                i => { items.splice(i, 1); ui.touch(); ui.update(); },
                {
                    isValid: V.isRuleComplete,
                    addDisabled: !functionEnabled('addRuleButtonEnabled'),
                    deleteDisabled: !functionEnabled('deleteRuleButtonEnabled'),
                    canDelete: () => true
                }),
            h('div', { class: 'grow' }, items.length ? ruleEditor(flow, items[sel], ui) : h('div', { class: 'muted' }, 'No rules.'))
        ),
        templatesEditor(flow, ui)
    );
}
